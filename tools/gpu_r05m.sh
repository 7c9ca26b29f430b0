#!/bin/bash
# Round-5 pass m: same-box A/B of k_bounds on the side stream beside k_hild at configs[2]
# (MPCEKF_BOUNDS_SIDE above the batch) against the default (serial above 16,384 cells), three
# interleaved pairs at 65,536 cells and one at 131,072.
#   gpurun --timeout 900 -- 'bash tools/gpu_r05m.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05m}
O=gpurun_out/$TAG
mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu"
for rep in 1 2 3; do
  $B > $O/bench_serial_$rep.json 2> $O/bench_serial_$rep.err || exit 1
  MPCEKF_BOUNDS_SIDE=10000000 $B > $O/bench_side_$rep.json 2> $O/bench_side_$rep.err || exit 1
done
$B --cells-per-gpu 131072 > $O/bench_131072_serial.json 2> $O/bench_131072_serial.err || exit 1
MPCEKF_BOUNDS_SIDE=10000000 $B --cells-per-gpu 131072 > $O/bench_131072_side.json 2> $O/bench_131072_side.err || exit 1
