#!/bin/bash
# Wide-path check on the GPU box: the whole -m gpu suite, then the configs[4] bench over
# the steady-state window under a kernel trace.  Usage: gpurun -- 'bash tools/wide_pass.sh TAG'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- \
  python3 bench.py --no-cpu --np 20 --nc 10 > $O/bench_wide.json 2> $O/bench_wide.err
