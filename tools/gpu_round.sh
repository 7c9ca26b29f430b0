#!/bin/bash
# The one GPU-box pass script (round 6; replaces the per-pass tools/gpu_r0*.sh).  Every
# step runs under its own time limit and the steps are chained: the first failure ends
# the call.  Output under gpurun_out/TAG/.
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh MODE TAG [pytest selection]'
# MODE:
#   tests    the -m gpu suite (optionally a selection) and the smoke
#   bench    the headline lines: configs[2] (default bench, steps 10-1010), configs[1],
#            configs[4], the 131,072-cell per-GPU load of configs[3], the v2-table line
#   trace    rocprofv3 kernel trace + stats of the default bench and of configs[1] / [4]
#   pmc      PMC traffic (tools/profile.sh) and SQ counters (tools/cell_pmc.sh) of the
#            default bench, then the bench line with that traffic attached (the Np = 20 pass:
#            PMCARGS="--np 20" bash tools/profile.sh TAG_np20 --np 20 --nc 10, in a call of its
#            own: its counter passes print nothing for minutes)
#   dropin   the C-ABI stage route at 65,536 and 1,024 cells (tools/dropin_bench.py: through
#            mpcekf.py, and driven from C with fresh or reused host buffers; sync and _async)
#   closing  tests + smoke + bench + trace + pmc + dropin on one build (the round's record)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
MODE=${1:-tests}
TAG=${2:-r06}
shift 2
SEL=${*:-tests}
O=gpurun_out/$TAG
mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu"

do_tests() {
  timeout -k 10 800 python -u -m pytest $SEL -x -v -m gpu --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
}
do_bench() {
  $B > $O/bench_default.json 2> $O/bench_default.err && \
  $B --cells-per-gpu 1024 > $O/bench_1024.json 2> $O/bench_1024.err && \
  $B --np 20 --nc 10 > $O/bench_wide.json 2> $O/bench_wide.err && \
  $B --cells-per-gpu 131072 > $O/bench_131072.json 2> $O/bench_131072.err && \
  $B --rom-lookup linear > $O/bench_linear.json 2> $O/bench_linear.err
}
do_trace() {
  for a in "default:" "1024:--cells-per-gpu 1024" "wide:--np 20 --nc 10"; do
    nm=${a%%:*}; args=${a#*:}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$nm -o run -- \
      python3 bench.py --no-cpu $args > $O/bench_trace_$nm.json 2> $O/bench_trace_$nm.err || return 1
  done
}
do_pmc() {
  bash tools/profile.sh $TAG && \
  bash tools/cell_pmc.sh $TAG && \
  timeout -k 10 300 python bench.py --pmc gpurun_out/prof_$TAG/pmc_traffic.json > $O/bench_pmc.json 2> $O/bench_pmc.err
}
do_dropin() {
  for rt in capi capi-async c c-async c-reuse c-async-reuse; do
    timeout -k 10 300 python tools/dropin_bench.py --route $rt --cells 65536 --steps 20 > $O/dropin_${rt}_65536.json \
      2> $O/dropin_${rt}_65536.err && \
    timeout -k 10 300 python tools/dropin_bench.py --route $rt --cells 1024 --steps 40 > $O/dropin_${rt}_1024.json \
      2> $O/dropin_${rt}_1024.err || return 1
  done
}
case $MODE in
  tests) do_tests ;;
  bench) do_bench ;;
  trace) do_trace ;;
  pmc) do_pmc ;;
  dropin) do_dropin ;;
  closing) do_tests && do_bench && do_trace && do_pmc && do_dropin ;;
  *) echo "unknown mode $MODE" >&2; exit 2 ;;
esac
