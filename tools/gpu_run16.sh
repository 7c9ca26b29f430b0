set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/dump_hild.py 650 /tmp/hild650.bin > gpurun_out/dump650.log 2>&1 && \
timeout -k 10 300 python tools/dump_hild.py 850 /tmp/hild850.bin > gpurun_out/dump850.log 2>&1 && \
timeout -k 10 200 ./tools/micro/hild_micro --ab 5 tools/micro/state450.bin /tmp/hild650.bin /tmp/hild850.bin > gpurun_out/ab5.log 2>&1
