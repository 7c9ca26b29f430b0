#!/bin/bash
# Same-box A/B of library builds on the bench (no CPU leg): each lib in turn, twice,
# alternating.  gpurun -- 'bash tools/ab_libs.sh TAG "BENCH ARGS" lib1.so lib2.so ...'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    MPCEKF_LIB=$L timeout -k 10 300 python bench.py --no-cpu $ARGS > $O/${n}_$rep.json 2> $O/${n}_$rep.err || exit 1
  done
done
python3 - $O "$@" <<'PY'
import json, os, sys
O = sys.argv[1]
for L in sys.argv[2:]:
    n = os.path.basename(L)[:-3]
    for rep in (1, 2):
        d = json.loads(open(f"{O}/{n}_{rep}.json").read().strip().split("\n")[-1])
        print(f"{n:22s} rep{rep} value {d['value'] / 1e6:8.2f}M  " +
              " ".join(f"{k} {v['ms_per_launch'] * 1e3:7.1f}" for k, v in d["kernels"].items()))
PY
