#!/bin/bash
# configs[4] (Np = 20 / Nc = 10) counter evidence on the current build: HBM traffic and
# FP64 work (tools/profile.sh's passes, reduced to pmc_traffic_np20.json, which bench.py
# attaches at --np 20 when the build id matches) and the SQ issue / wait / LDS picture
# of the dominant kernels (pmc_sq_np20.json).  One counter group per rocprofv3 pass.
# Usage (GPU box): bash tools/wide_pmc.sh TAG [bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-wide}
shift
ARGS=${*:---steps 200 --warmup 400}
O=gpurun_out/wpmc_$TAG
mkdir -p $O
run() {  # name counters...
  local nm=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -f csv -d $O/$nm -o run -- \
    python3 bench.py --no-cpu --np 20 --nc 10 $ARGS > $O/$nm.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run fp64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 && \
python3 tools/pmc_traffic.py $O --np 20 --steps $(echo $ARGS | sed -n 's/.*--steps \([0-9]*\).*/\1/p') > $O/pmc_traffic_np20.json && \
run a SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run b SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run c SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM && \
run e SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS && \
python3 tools/pmc_sq.py $O/pmc_sq_np20.json $O/a $O/b $O/c $O/e
