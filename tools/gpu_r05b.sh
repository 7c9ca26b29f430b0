#!/bin/bash
# Round-5 second GPU pass: v3 lookups compiled per instantiation (linear kernels = the
# round-4 code), interleaved polynomial rows, T-invariant rows; the device-resident stage
# route.  GPU tests (new files first, then the suite), configs[2] linear / quintic,
# configs[1] / configs[4] quintic, kernel traces of both lookups, drop-in routes.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05b.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05b}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_handles.py tests/test_gpu_stage_route.py > $O/gpu_new.log 2>&1 || exit 1
timeout -k 10 600 $T -m gpu tests --ignore=tests/test_gpu_handles.py --ignore=tests/test_gpu_stage_route.py \
  > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
$B --rom-lookup linear > $O/bench_linear.json 2> $O/bench_linear.err || exit 1
$B --rom-lookup quintic > $O/bench_quintic.json 2> $O/bench_quintic.err || exit 1
$B --rom-lookup quintic --cells-per-gpu 1024 > $O/bench_quintic_1024.json 2> $O/bench_quintic_1024.err || exit 1
$B --rom-lookup quintic --np 20 --nc 10 > $O/bench_quintic_wide.json 2> $O/bench_quintic_wide.err || exit 1
for lk in linear quintic; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$lk -o run -- \
    python3 bench.py --no-cpu --rom-lookup $lk --steps 300 > $O/bench_trace_$lk.json 2> $O/bench_trace_$lk.err || exit 1
done
D="timeout -k 10 300 python tools/dropin_bench.py"
$D --route capi --cells 65536 --steps 20 > $O/dropin_capi_65536.json 2> $O/dropin_capi_65536.err || exit 1
$D --route device --cells 65536 --steps 20 > $O/dropin_device_65536.json 2> $O/dropin_device_65536.err || exit 1
$D --route host --cells 65536 --steps 20 > $O/dropin_host_65536.json 2> $O/dropin_host_65536.err || exit 1
$D --route capi --cells 1024 --steps 40 > $O/dropin_capi_1024.json 2> $O/dropin_capi_1024.err || exit 1
$D --route device --cells 1024 --steps 40 > $O/dropin_device_1024.json 2> $O/dropin_device_1024.err
