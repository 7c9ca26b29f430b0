#!/bin/bash
# Round-4 closing GPU pass on the current build: the GPU suite, the bench lines
# (configs[2] with the CPU leg, full charge, configs[1], configs[3] per-GPU load,
# configs[4]), the rocprofv3 kernel trace + PMC traffic of the default and the configs[4]
# bench (stamped lines after), the Np = 5 SQ counters, the k_cell section stamps and the
# MATLAB drop-in route.  Every step has its own time limit; the first failure ends it.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r04_final.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04z}
O=gpurun_out/$TAG
mkdir -p $O
B="timeout -k 10 300 python bench.py"
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
$B > $O/bench.json 2> $O/bench.err || exit 1
$B --no-cpu --steps 3001 --warmup 0 > $O/bench_full_charge.json 2> $O/bench_full_charge.err || exit 1
$B --no-cpu --cells-per-gpu 1024 > $O/bench_1024.json 2> $O/bench_1024.err || exit 1
$B --no-cpu --cells-per-gpu 131072 > $O/bench_131072.json 2> $O/bench_131072.err || exit 1
$B --no-cpu --np 20 --nc 10 > $O/bench_wide.json 2> $O/bench_wide.err || exit 1
bash tools/profile.sh $TAG || exit 1
$B --pmc gpurun_out/prof_$TAG/pmc_traffic.json > $O/bench_stamped.json 2> $O/bench_stamped.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/wide_trace -o run -- \
  python3 bench.py --no-cpu --np 20 --nc 10 > $O/bench_wide_under_trace.json 2> $O/bench_wide_under_trace.err || exit 1
bash tools/wide_pmc.sh $TAG --steps 200 --warmup 400 || exit 1
$B --no-cpu --np 20 --nc 10 --pmc gpurun_out/wpmc_$TAG/pmc_traffic_np20.json > $O/bench_wide_stamped.json \
  2> $O/bench_wide_stamped.err || exit 1
bash tools/cell_pmc.sh $TAG || exit 1
if [ -f mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so ]; then
  MPCEKF_LIB=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so timeout -k 10 300 python tools/stamps.py 65536 300 \
    > $O/stamps_65536.txt 2>&1 || exit 1
fi
timeout -k 10 300 python tools/dropin_bench.py --cells 1024 --steps 40 > $O/dropin_1024.json 2> $O/dropin_1024.err || exit 1
timeout -k 10 300 python tools/dropin_bench.py --cells 65536 --steps 20 > $O/dropin_65536.json 2> $O/dropin_65536.err
