set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/w3
timeout -k 10 300 python bench.py --np 20 --nc 10 --no-cpu > gpurun_out/w3/bench_wide.json 2> gpurun_out/w3/bench_wide.err
