#!/bin/bash
# configs[1] (1,024 cells) under a kernel trace: the default path and the lane-quad EKF
# (MPCEKF_QUAD=1).  Usage (GPU box): bash tools/small_batch.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default -o run -- \
  python3 bench.py --no-cpu --cells-per-gpu 1024 > $O/default.json 2> $O/default.err && \
MPCEKF_QUAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/quad -o run -- \
  python3 bench.py --no-cpu --cells-per-gpu 1024 > $O/quad.json 2> $O/quad.err && \
timeout -k 10 300 python3 bench.py --no-cpu --cells-per-gpu 1024 > $O/plain.json 2> $O/plain.err
