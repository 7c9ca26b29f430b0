#!/bin/bash
# Round-4 closing evidence on the final build: tools/gpu_r04_final.sh, then the
# 1,048,576-cell configs[3] input as one context and the gloo coordinator at world size 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04r}
O=gpurun_out/$TAG
bash tools/gpu_r04_final.sh $TAG || exit 1
timeout -k 10 300 python bench.py --no-cpu --total-cells 1048576 > $O/bench_1048576_one_gpu.json 2> $O/bench_1048576_one_gpu.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --force-dist > $O/bench_gloo_world1.json 2> $O/bench_gloo_world1.err
