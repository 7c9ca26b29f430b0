#!/bin/bash
# Round-5 pass e: small batches spread one wave per CU (spread_block) — GPU tests, then a
# same-box A/B of MPCEKF_SPREAD=0/1 at 1,024 / 4,096 / 16,384 / 65,536 cells (quintic
# tables), kernel traces at 1,024 cells, and k_cell section stamps linear vs quintic.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05e.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05e}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
for n in 1024 4096 16384 65536; do
  for sp in 0 1; do
    MPCEKF_SPREAD=$sp $B --cells-per-gpu $n > $O/bench_${n}_spread$sp.json 2> $O/bench_${n}_spread$sp.err || exit 1
  done
done
for sp in 0 1; do
  MPCEKF_SPREAD=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_1024_spread$sp -o run -- \
    python3 bench.py --no-cpu --cells-per-gpu 1024 --steps 300 > $O/bench_trace_1024_spread$sp.json \
    2> $O/bench_trace_1024_spread$sp.err || exit 1
done
V=mpc-ekf4fastcharge_amd/_build/libmpcekf_plu.so
if [ -f $V ]; then  # the one-path v3 lookup (MPCEKF_PL_UNIFIED=1) against the default, same box
  for rep in 1 2; do
    $B > $O/bench_main_$rep.json 2> $O/bench_main_$rep.err || exit 1
    MPCEKF_LIB=$V $B > $O/bench_plu_$rep.json 2> $O/bench_plu_$rep.err || exit 1
  done
fi
S=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so
if [ -f $S ]; then
  for lk in linear quintic; do
    MPCEKF_LIB=$S timeout -k 10 300 python tools/stamps.py 65536 300 $lk > $O/stamps_65536_$lk.txt 2>&1 || exit 1
  done
fi
timeout -k 10 300 python tools/dropin_probe.py 65536 6 > $O/dropin_probe.jsonl 2> $O/dropin_probe.err || exit 1
