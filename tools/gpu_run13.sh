set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
