set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/w1
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -v --timeout 200 --timeout-method thread > gpurun_out/w1/wide_tests.log 2>&1
