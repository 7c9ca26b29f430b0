#!/bin/bash
# Np = 5 SQ issue / wait / LDS picture of the bench kernels (k_cell, k_hild, k_plant,
# k_bounds) on the current build, one counter group per rocprofv3 pass, reduced by
# tools/pmc_sq.py.  Usage (GPU box): bash tools/cell_pmc.sh TAG [bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-np5}
shift
ARGS=${*:---steps 200 --warmup 10}
O=gpurun_out/cpmc_$TAG
mkdir -p $O
run() {  # name counters...
  local nm=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -f csv -d $O/$nm -o run -- \
    python3 bench.py --no-cpu $ARGS > $O/$nm.log 2>&1
}
run a SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run b SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run c SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM && \
run e SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR && \
python3 tools/pmc_sq.py $O/pmc_sq_np5.json $O/a $O/b $O/c $O/e
