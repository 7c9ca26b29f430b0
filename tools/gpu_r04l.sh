#!/bin/bash
# Round-4 extra lines on the current build: the new edge-record tests, the 1,048,576-cell
# configs[3] input as one context on one GPU, the gloo timing coordinator at world size 1,
# and the default bench again (box-to-box spread).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -x -v -m gpu -k "edge_records or side_stream" \
  --timeout 200 --timeout-method thread > $O/tests_edge.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu --total-cells 1048576 --steps 200 --warmup 10 > $O/bench_1048576_one_gpu.json 2> $O/bench_1048576_one_gpu.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --force-dist > $O/bench_gloo_world1.json 2> $O/bench_gloo_world1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu > $O/bench_again.json 2> $O/bench_again.err
