#!/bin/bash
# One GPU-box pass: parity tests, the default bench line (with the CPU baseline),
# then the rocprofv3 kernel trace of the same bench command.
#   gpurun --timeout 1100 -- 'bash tools/gpu_pass.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 bench.py --no-cpu > $O/bench_under_trace.json 2> $O/bench_under_trace.err
