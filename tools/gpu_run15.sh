set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 ./tools/micro/hild_micro --ab 5 tools/micro/stateA.bin tools/micro/state450.bin > gpurun_out/ab4.log 2>&1 && \
timeout -k 10 300 python tools/diag_hild.py 65536 1010 gpurun_out/diag_hild.json > gpurun_out/diag_hild.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1
