#!/bin/bash
# Round-4 GPU pass: the GPU suite, the default bench line (CPU leg included), a same-box
# A/B of library variants on the bench, and the MATLAB drop-in stage route.
#   gpurun --timeout 1100 -- 'bash tools/gpu_r04.sh TAG "BENCH ARGS" variant1.so ...'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
if [ $# -gt 0 ]; then
  bash tools/ab_libs.sh $TAG/ab "$ARGS" mpc-ekf4fastcharge_amd/_build/libmpcekf.so "$@" > $O/ab.txt 2>&1 || exit 1
fi
timeout -k 10 300 python tools/dropin_bench.py --cells 1024 --steps 40 > $O/dropin_1024.json 2> $O/dropin_1024.err || exit 1
timeout -k 10 300 python tools/dropin_bench.py --cells 65536 --steps 20 > $O/dropin_65536.json 2> $O/dropin_65536.err || exit 1
