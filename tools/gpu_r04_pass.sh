#!/bin/bash
# Round-4 GPU pass on the current build: the GPU suite, the default bench line (CPU leg
# included), a same-box A/B against variant libraries, k_cell / k_plant section stamps,
# and the rocprofv3 kernel trace + PMC traffic of the default bench command.
#   gpurun --timeout 1100 -- 'ENV_AB="VAR=value" bash tools/gpu_r04_pass.sh TAG [variant.so ...]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
if [ $# -gt 0 ]; then
  bash tools/ab_libs.sh $TAG/ab "" mpc-ekf4fastcharge_amd/_build/libmpcekf.so "$@" > $O/ab.txt 2>&1 || exit 1
fi
if [ -n "$WIDE_AB" ]; then  # configs[4]: A/B against variant libraries, kernel trace + traffic of the product library
  bash tools/ab_libs.sh $TAG/ab_wide "--np 20 --nc 10" mpc-ekf4fastcharge_amd/_build/libmpcekf.so $WIDE_AB > $O/ab_wide.txt 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/wide_trace -o run -- \
    python3 bench.py --no-cpu --np 20 --nc 10 > $O/bench_wide_under_trace.json 2> $O/bench_wide_under_trace.err || exit 1
  bash tools/wide_pmc.sh $TAG --steps 200 --warmup 400 || exit 1
fi
if [ -n "$ENV_AB" ]; then  # the product library under an environment override, twice
  for rep in 1 2; do
    env $ENV_AB timeout -k 10 300 python bench.py --no-cpu > $O/env_ab_$rep.json 2> $O/env_ab_$rep.err || exit 1
  done
fi
if [ -f mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so ]; then
  for N in 65536 1024; do
    MPCEKF_LIB=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so timeout -k 10 300 python tools/stamps.py $N 300 > $O/stamps_$N.txt 2>&1 || exit 1
  done
fi
bash tools/profile.sh $TAG || exit 1
timeout -k 10 300 python bench.py --no-cpu --pmc gpurun_out/prof_$TAG/pmc_traffic.json > $O/bench_stamped.json 2> $O/bench_stamped.err
