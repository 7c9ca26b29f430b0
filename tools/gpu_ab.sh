#!/bin/bash
# A/B of environment variants on the default bench (no CPU leg), after the GPU tests.
#   gpurun -- 'bash tools/gpu_ab.sh TAG "ENV1" "ENV2" ...'   (ENV: space-separated VAR=value, or "-")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
i=0
for V in "$@"; do
  i=$((i+1))
  if [ "$V" = "-" ]; then V=""; fi
  env $V timeout -k 10 300 python bench.py --no-cpu $BENCH_ARGS > $O/ab_$i.json 2> $O/ab_$i.err || exit 1
  echo "$V" > $O/ab_$i.env
done
