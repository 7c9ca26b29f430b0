#!/bin/bash
# Round-5 closing pass i (headline, one build id): GPU tests and smoke, the default bench's rocprof profile and PMC traffic
# (tools/profile.sh), the default bench line with the CPU leg and that traffic, its kernel
# trace, configs[1] / configs[4] / the linear-table line, the C-ABI stage route.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05i.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05i}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash tools/profile.sh $TAG || exit 1
timeout -k 10 300 python bench.py --pmc gpurun_out/prof_$TAG/pmc_traffic.json > $O/bench_default.json 2> $O/bench_default.err || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_default -o run -- \
  python3 bench.py --no-cpu > $O/bench_trace_default.json 2> $O/bench_trace_default.err || exit 1
$B --cells-per-gpu 1024 > $O/bench_1024.json 2> $O/bench_1024.err || exit 1
$B --cells-per-gpu 131072 > $O/bench_131072.json 2> $O/bench_131072.err || exit 1
$B --rom-lookup linear > $O/bench_linear.json 2> $O/bench_linear.err || exit 1
$B --np 20 --nc 10 > $O/bench_wide.json 2> $O/bench_wide.err || exit 1
timeout -k 10 300 python tools/dropin_bench.py --route capi --cells 65536 --steps 20 > $O/dropin_capi_65536.json \
  2> $O/dropin_capi_65536.err || exit 1
bash tools/cell_pmc.sh $TAG || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
$B --total-cells 1048576 > $O/bench_1048576_one_gpu.json 2> $O/bench_1048576_one_gpu.err || exit 1
$B --warmup 0 --steps 3001 > $O/bench_full_charge.json 2> $O/bench_full_charge.err || exit 1
timeout -k 10 300 python tools/dropin_bench.py --route capi --cells 1024 --steps 40 > $O/dropin_capi_1024.json \
  2> $O/dropin_capi_1024.err || exit 1
S=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so
for lk in linear quintic; do
  MPCEKF_LIB=$S timeout -k 10 300 python tools/stamps.py 65536 300 $lk > $O/stamps_65536_$lk.txt 2>&1 || exit 1
done
