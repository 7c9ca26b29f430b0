#!/bin/bash
# Round-5 pass j: the plant inside the lane-quad k_ekf4 (quad_plant) — GPU tests, then a same-box
# A/B at 1,024 / 4,096 / 8,192 cells of the lane per cell path (MPCEKF_QUAD=0) against the quad
# default, and a kernel trace at 1,024 cells.
#   gpurun --timeout 900 -- 'bash tools/gpu_r05j.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05j}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
for n in 1024 4096 8192; do
  MPCEKF_QUAD=0 $B --cells-per-gpu $n > $O/bench_${n}_cell.json 2> $O/bench_${n}_cell.err || exit 1
  $B --cells-per-gpu $n > $O/bench_${n}_quad.json 2> $O/bench_${n}_quad.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_1024 -o run -- \
  python3 bench.py --no-cpu --cells-per-gpu 1024 --steps 300 > $O/bench_trace_1024.json 2> $O/bench_trace_1024.err || exit 1
