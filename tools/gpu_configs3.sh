#!/bin/bash
# configs[3] on one GPU: the eight-shard + single-context parity test, then bench lines
# for one 131,072-cell shard over the steady-state window and for the whole
# 1,048,576-cell input as one context.  Usage: gpurun -- 'bash tools/gpu_configs3.sh TAG'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs3.py -x -v -m gpu --timeout 350 --timeout-method thread > $O/configs3_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --cells-per-gpu 131072 --steps 1000 > $O/bench_131072.json 2> $O/bench_131072.err && \
timeout -k 10 200 python bench.py --no-cpu --total-cells 1048576 --steps 1000 > $O/bench_1048576_one_gpu.json 2> $O/bench_1048576_one_gpu.err
