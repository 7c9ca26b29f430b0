#!/bin/bash
# Round-5 pass e: GPU tests, then same-box A/Bs of the small-batch mappings at 1,024 /
# 4,096 / 16,384 cells (quintic tables): the packed launch (MPCEKF_SPREAD=0), one wave per CU
# (spread, the default) and the spread lane-quad iterEKF (MPCEKF_QUAD=1, k_ekf4 at 512
# registers); kernel traces at 1,024 cells; configs[2] quintic / linear; k_cell section
# stamps linear vs quintic; the drop-in stall probe.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05e.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05e}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
for n in 1024 4096 16384; do
  MPCEKF_SPREAD=0 $B --cells-per-gpu $n > $O/bench_${n}_packed.json 2> $O/bench_${n}_packed.err || exit 1
  $B --cells-per-gpu $n > $O/bench_${n}_spread.json 2> $O/bench_${n}_spread.err || exit 1
  MPCEKF_QUAD=1 $B --cells-per-gpu $n > $O/bench_${n}_quad.json 2> $O/bench_${n}_quad.err || exit 1
done
for v in packed spread quad; do
  E="MPCEKF_NONE=0"
  [ $v = packed ] && E="MPCEKF_SPREAD=0"
  [ $v = quad ] && E="MPCEKF_QUAD=1"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_1024_$v -o run -- \
    python3 bench.py --no-cpu --cells-per-gpu 1024 --steps 300 > $O/bench_trace_1024_$v.json \
    2> $O/bench_trace_1024_$v.err || exit 1
done
$B > $O/bench_65536.json 2> $O/bench_65536.err || exit 1
$B --rom-lookup linear > $O/bench_65536_linear.json 2> $O/bench_65536_linear.err || exit 1
S=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so
for lk in linear quintic; do
  MPCEKF_LIB=$S timeout -k 10 300 python tools/stamps.py 65536 300 $lk > $O/stamps_65536_$lk.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/dropin_probe.py 65536 6 > $O/dropin_probe.jsonl 2> $O/dropin_probe.err || exit 1
