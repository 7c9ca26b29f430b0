#!/bin/bash
# Same-box A/B of the rolling flush schedule (MPCEKF_FLUSH_ROLL=1, default) against every
# cell flushed at once each 32 steps (=0): the bench twice each, alternating.
#   gpurun -- 'bash tools/roll_ab.sh TAG "BENCH ARGS"'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; ARGS=$2
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for R in 1 0; do
    MPCEKF_FLUSH_ROLL=$R timeout -k 10 300 python bench.py --no-cpu $ARGS > $O/roll${R}_$rep.json 2> $O/roll${R}_$rep.err || exit 1
  done
done
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
for rep in (1, 2):
    for R in (1, 0):
        d = json.loads(open(f"{O}/roll{R}_{rep}.json").read().strip().split("\n")[-1])
        print(f"roll={R} rep{rep} value {d['value'] / 1e6:8.2f}M ms/step {d['ms_per_step']:.4f} " +
              " ".join(f"{k} {v['ms_per_launch'] * 1e3:7.1f}" for k, v in d["kernels"].items()))
PY
