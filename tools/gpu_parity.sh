set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo | grep -m2 gfx > gpurun_out/info.txt || true
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu1.log 2>&1
