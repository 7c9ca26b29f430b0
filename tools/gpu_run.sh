#!/bin/bash
# One GPU-box pass: parity tests, k_cell section stamps, the default bench line.
#   gpurun --timeout 1100 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
MPCEKF_LIB=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1
