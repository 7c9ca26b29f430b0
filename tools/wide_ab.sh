#!/bin/bash
# Wide-horizon (configs[4]) bench of the default library and its A/B variants under a
# kernel trace.  Usage (GPU box): bash tools/wide_ab.sh TAG [variant ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for V in default "$@"; do
  if [ "$V" = default ]; then L=""; else L=mpc-ekf4fastcharge_amd/_build/libmpcekf_$V.so; fi
  MPCEKF_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$V -o run -- \
    python3 bench.py --no-cpu --np 20 --nc 10 $BENCH_ARGS > $O/$V.json 2> $O/$V.err || exit 1
done
