#!/bin/bash
# The -m gpu suite on the box (one process), log under gpurun_out/TAG/.
# Usage: gpurun -- 'bash tools/gpu_tests.sh TAG [pytest selection]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${*:-tests} -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
