#!/bin/bash
# Round-5 pass t: k_hild_wide's group LDS stride padded 516 -> 520 doubles (a scratch build,
# _build/libmpcekf_pad.so): the Np = 20 GPU tests on it, its SQ LDS counters,
# then a same-box A/B against the product library at configs[4], two interleaved pairs.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05t.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05t}
O=gpurun_out/$TAG
mkdir -p $O
PAD=mpc-ekf4fastcharge_amd/_build/libmpcekf_pad.so
MAIN=mpc-ekf4fastcharge_amd/_build/libmpcekf.so
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
MPCEKF_LIB=$PAD timeout -k 10 600 $T -m gpu tests/test_gpu_wide.py tests/test_gpu_horizons.py > $O/gpu_tests_pad.log 2>&1 || exit 1
for v in main pad; do
  L=$MAIN; [ $v = pad ] && L=$PAD
  MPCEKF_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
    -f csv -d $O/lds_$v -o run -- python3 bench.py --no-cpu --np 20 --nc 10 --steps 200 --warmup 400 > $O/lds_$v.log 2>&1 || exit 1
done
B="timeout -k 10 300 python bench.py --no-cpu --np 20 --nc 10"
for rep in 1 2; do
  for v in main pad; do
    L=$MAIN; [ $v = pad ] && L=$PAD
    MPCEKF_LIB=$L $B > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || exit 1
  done
done
