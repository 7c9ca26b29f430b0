#!/bin/bash
# Same-box A/B of one environment override on the bench (no CPU leg), alternating, twice,
# at each batch size.  gpurun -- 'bash tools/env_ab.sh TAG VAR=value "CELLS..." [bench args]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; OVR=$2; CELLS=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
for N in $CELLS; do
  for rep in 1 2; do
    timeout -k 10 300 python bench.py --no-cpu --cells-per-gpu $N "$@" > $O/base_${N}_$rep.json 2> $O/base_${N}_$rep.err || exit 1
    env $OVR timeout -k 10 300 python bench.py --no-cpu --cells-per-gpu $N "$@" > $O/ovr_${N}_$rep.json \
      2> $O/ovr_${N}_$rep.err || exit 1
  done
done
python3 - $O "$OVR" $CELLS <<'PY'
import json, sys
O, ovr = sys.argv[1], sys.argv[2]
for N in sys.argv[3:]:
    for arm in ("base", "ovr"):
        for rep in (1, 2):
            d = json.loads(open(f"{O}/{arm}_{N}_{rep}.json").read().strip().split("\n")[-1])
            print(f"{N:>7} {arm if arm == 'base' else ovr:28s} rep{rep} value {d['value'] / 1e6:9.3f}M  ms/step "
                  f"{d['ms_per_step'] * 1e3:7.1f} us  " +
                  " ".join(f"{k} {v['ms_per_launch'] * 1e3:6.1f}" for k, v in d["kernels"].items()))
PY
