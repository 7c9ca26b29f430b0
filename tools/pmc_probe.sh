#!/bin/bash
# Quick SQ counter passes over a short bench (issue/wait/LDS picture per kernel).
# Usage (on the GPU box): bash tools/pmc_probe.sh TAG [bench.py args]   (MPCEKF_LIB selects a variant)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-probe}
shift
ARGS=${*:---steps 64 --warmup 4}
O=gpurun_out/pmc_$TAG
mkdir -p $O
run() {  # name counters...
  local nm=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" -f csv -d $O/$nm -o run -- \
    python3 bench.py --no-cpu $ARGS > $O/$nm.log 2>&1
}
run a SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run b SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run c SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM && \
run d GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS && \
run e SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
