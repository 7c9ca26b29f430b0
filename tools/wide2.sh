set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/w2
timeout -k 10 200 python -u tools/diag_wide.py > gpurun_out/w2/diag.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/w2/trace -o run -- \
  python3 bench.py --np 20 --nc 10 --steps 300 --no-cpu > gpurun_out/w2/bench_wide.json 2> gpurun_out/w2/bench_wide.err
