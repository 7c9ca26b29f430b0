#!/bin/bash
# rocprofv3 evidence for the bench on the current build: kernel trace + stats, then one
# PMC pass per counter group (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass;
# MI355X_MICROARCH.md), reduced by tools/pmc_traffic.py into a JSON stamped with the
# library's build id (bench.py attaches traffic only when the ids match).
# Usage (on the GPU box): bash tools/profile.sh TAG [extra bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
shift
EXTRA="$*"
O=gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 bench.py --no-cpu $EXTRA > $O/bench_under_trace.json 2> $O/bench_under_trace.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- \
  python3 bench.py --no-cpu $EXTRA > $O/bench_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- \
  python3 bench.py --no-cpu $EXTRA > $O/bench_write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
  -f csv -d $O/fp64 -o run -- python3 bench.py --no-cpu $EXTRA > $O/bench_fp64.log 2>&1 && \
python3 tools/pmc_traffic.py $O $PMCARGS > $O/pmc_traffic.json
