set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/d1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -v --timeout 200 --timeout-method thread > gpurun_out/d1/tests.log 2>&1
