#!/bin/bash
# One GPU-box pass: parity tests, the default bench line (with the CPU baseline), the
# full 3001-step charge, configs[1] and configs[4] bench lines, then the rocprofv3
# kernel trace + PMC passes of the default bench command (tools/profile.sh), the bench
# line again with that PMC file attached, and the configs[4] counters (tools/wide_pmc.sh).
#   gpurun --timeout 1100 -- 'bash tools/gpu_pass.sh TAG [quick]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
( [ "$2" = "quick" ] || (
timeout -k 10 300 python bench.py --no-cpu --steps 3001 --warmup 0 > $O/bench_full_charge.json 2> $O/bench_full_charge.err && \
timeout -k 10 300 python bench.py --no-cpu --cells-per-gpu 1024 > $O/bench_1024.json 2> $O/bench_1024.err && \
timeout -k 10 300 python bench.py --no-cpu --np 20 --nc 10 > $O/bench_wide.json 2> $O/bench_wide.err && \
bash tools/profile.sh $TAG && \
timeout -k 10 300 python bench.py --pmc gpurun_out/prof_$TAG/pmc_traffic.json > $O/bench_stamped.json 2> $O/bench_stamped.err && \
bash tools/wide_pmc.sh $TAG && \
timeout -k 10 300 python bench.py --no-cpu --np 20 --nc 10 --pmc gpurun_out/wpmc_$TAG/pmc_traffic_np20.json \
  > $O/bench_wide_stamped.json 2> $O/bench_wide_stamped.err ) )
