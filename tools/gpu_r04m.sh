#!/bin/bash
# Round-4 pass after the register pivot search in lu_solve_n: the closing pass
# (tools/gpu_r04_final.sh) on the new build, then a same-box A/B of configs[4] against the
# scratch-pivot build, the 1,048,576-cell configs[3] input as one context over 1000 steps
# and the gloo timing coordinator at world size 1 outside a launcher.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04m}
O=gpurun_out/$TAG
bash tools/gpu_r04_final.sh $TAG || exit 1
bash tools/ab_libs.sh $TAG/ab_wide "--np 20 --nc 10" mpc-ekf4fastcharge_amd/_build/libmpcekf.so \
  mpc-ekf4fastcharge_amd/_build/libmpcekf_lu0.so > $O/ab_wide_lu.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu --total-cells 1048576 > $O/bench_1048576_one_gpu.json 2> $O/bench_1048576_one_gpu.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --force-dist > $O/bench_gloo_world1.json 2> $O/bench_gloo_world1.err
