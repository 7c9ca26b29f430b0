set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -s > gpurun_out/pytest_gpu2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu > gpurun_out/bench2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu --bounds 0 >> gpurun_out/bench2.log 2>&1
