set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python tools/dump_hild.py 650 /tmp/hild650.bin > gpurun_out/dump650.log 2>&1 && \
HILD_T=0 timeout -k 10 200 ./tools/micro/hild_micro --ab 5 tools/micro/stateA.bin tools/micro/state450.bin /tmp/hild650.bin > gpurun_out/ab_lr.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1
