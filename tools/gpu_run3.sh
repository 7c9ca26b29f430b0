set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu3.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 && \
bash tools/profile.sh r01 && \
timeout -k 10 600 python bench.py > gpurun_out/bench3.log 2>&1
