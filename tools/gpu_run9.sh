set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/dump_hild.py 450 gpurun_out/hild450.bin > gpurun_out/dump.log 2>&1 && \
timeout -k 10 120 ./tools/micro/hild_micro --state gpurun_out/hild450.bin gpurun_out/probe450.bin > gpurun_out/replay.log 2>&1
