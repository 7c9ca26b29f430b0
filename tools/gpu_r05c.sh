#!/bin/bash
# Round-5 third GPU pass: FMA Horner, the k0 / Rf reuse across getVariables / getChatV /
# getChatZ / EKFmatsHandler, lin_fields by a gather kernel.  GPU tests (new files first),
# configs[2] linear / quintic with kernel traces, the default bench's rocprof profile with
# PMC traffic, the C-ABI stage route.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05c.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05c}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_handles.py tests/test_gpu_stage_route.py > $O/gpu_new.log 2>&1 || exit 1
timeout -k 10 600 $T -m gpu tests --ignore=tests/test_gpu_handles.py --ignore=tests/test_gpu_stage_route.py \
  > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
$B --rom-lookup linear > $O/bench_linear.json 2> $O/bench_linear.err || exit 1
$B --rom-lookup quintic > $O/bench_quintic.json 2> $O/bench_quintic.err || exit 1
for lk in linear quintic; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$lk -o run -- \
    python3 bench.py --no-cpu --rom-lookup $lk --steps 300 > $O/bench_trace_$lk.json 2> $O/bench_trace_$lk.err || exit 1
done
bash tools/profile.sh $TAG || exit 1
timeout -k 10 300 python bench.py --pmc gpurun_out/prof_$TAG/pmc_traffic.json > $O/bench_default.json 2> $O/bench_default.err || exit 1
D="timeout -k 10 300 python tools/dropin_bench.py"
$D --route capi --cells 65536 --steps 20 > $O/dropin_capi_65536.json 2> $O/dropin_capi_65536.err || exit 1
$D --route capi --cells 1024 --steps 40 > $O/dropin_capi_1024.json 2> $O/dropin_capi_1024.err
