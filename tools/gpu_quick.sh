set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q1
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/q1/bench.json 2> gpurun_out/q1/bench.err && \
timeout -k 10 200 python bench.py --no-cpu --cells-per-gpu 1024 > gpurun_out/q1/bench_1024.json 2> gpurun_out/q1/bench_1024.err && \
timeout -k 10 200 python bench.py --no-cpu --timing-every 1 > gpurun_out/q1/bench_every1.json 2> gpurun_out/q1/bench_every1.err
