set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/w5
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w5/wide_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/w5/trace -o run -- \
  python3 bench.py --np 20 --nc 10 --no-cpu > gpurun_out/w5/bench_wide.json 2> gpurun_out/w5/bench_wide.err
