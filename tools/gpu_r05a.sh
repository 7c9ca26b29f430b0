#!/bin/bash
# Round-5 first GPU pass: the ABI v3 electrode lookups (tests/test_gpu_handles.py), the
# whole GPU suite, and the configs[2] bench with the v2 linear and the v3 quintic tables.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05a.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05a}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_handles.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_handles.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  --ignore=tests/test_gpu_handles.py > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
$B --rom-lookup linear > $O/bench_linear.json 2> $O/bench_linear.err || exit 1
$B --rom-lookup quintic > $O/bench_quintic.json 2> $O/bench_quintic.err || exit 1
$B --rom-lookup quintic --np 20 --nc 10 > $O/bench_quintic_wide.json 2> $O/bench_quintic_wide.err
