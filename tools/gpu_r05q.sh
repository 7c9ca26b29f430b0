#!/bin/bash
# Round-5 pass q: same-box A/B of the theta-invariant lookups (istride 0; MPCEKF_THETA_CONST=0
# keeps the gather) at configs[2], two interleaved pairs, then the closing pass (tests, smoke,
# profile, PMC, bench lines, SQ counters, stamps) on the same build.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05q.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05q}
O=gpurun_out/$TAG
mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu"
for rep in 1 2; do
  MPCEKF_THETA_CONST=0 $B > $O/ab_gather_$rep.json 2> $O/ab_gather_$rep.err || exit 1
  $B > $O/ab_const_$rep.json 2> $O/ab_const_$rep.err || exit 1
done
bash tools/gpu_r05i.sh $TAG
