#!/bin/bash
# Round-5 pass s: the speculative next-row t in k_hild's fast sweep (a scratch build,
# _build/libmpcekf_spec.so) — the GPU parity suite on it, then a same-box
# A/B against the product library at configs[2] and configs[1], two interleaved pairs each.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05s.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05s}
O=gpurun_out/$TAG
mkdir -p $O
SPEC=mpc-ekf4fastcharge_amd/_build/libmpcekf_spec.so
MAIN=mpc-ekf4fastcharge_amd/_build/libmpcekf.so
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
MPCEKF_LIB=$SPEC timeout -k 10 700 $T -m gpu tests --ignore tests/test_gpu_wide.py > $O/gpu_tests_spec.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
for rep in 1 2; do
  for v in main spec; do
    L=$MAIN; [ $v = spec ] && L=$SPEC
    MPCEKF_LIB=$L $B > $O/ab_${v}_65536_$rep.json 2> $O/ab_${v}_65536_$rep.err || exit 1
    MPCEKF_LIB=$L $B --cells-per-gpu 1024 > $O/ab_${v}_1024_$rep.json 2> $O/ab_${v}_1024_$rep.err || exit 1
  done
done
