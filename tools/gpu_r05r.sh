#!/bin/bash
# Round-5 pass r: the two configurations below their review targets, on the final build —
# configs[1] (1,024 cells) and configs[4] (Np = 20 / Nc = 10): kernel traces, the wide
# counters (HBM traffic, FP64 work, SQ issue / wait) and the stamped wide bench line.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05r.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05r}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_1024 -o run -- \
  python3 bench.py --no-cpu --cells-per-gpu 1024 > $O/bench_trace_1024.json 2> $O/bench_trace_1024.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_wide -o run -- \
  python3 bench.py --no-cpu --np 20 --nc 10 > $O/bench_trace_wide.json 2> $O/bench_trace_wide.err || exit 1
bash tools/wide_pmc.sh $TAG || exit 1
timeout -k 10 300 python bench.py --no-cpu --np 20 --nc 10 --pmc gpurun_out/wpmc_$TAG/pmc_traffic_np20.json \
  > $O/bench_wide_stamped.json 2> $O/bench_wide_stamped.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --cells-per-gpu 1024 > $O/bench_1024.json 2> $O/bench_1024.err || exit 1
