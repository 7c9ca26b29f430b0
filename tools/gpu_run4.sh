set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu5.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu5.log
timeout -k 10 600 python bench.py > gpurun_out/bench5.log 2>&1
