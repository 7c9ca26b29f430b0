#!/bin/bash
# Round-5 pass g: the stage route's host copies through the pinned bounce buffer (Xfer) and
# the lane-quad small-batch default (MPCEKF_QUAD_MAX 8,192) — GPU tests; the drop-in probe
# with direct copies (MPCEKF_BOUNCE_MAX=0) and bounced; the C-ABI stage-route lines; the
# small-batch bench lines.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05g.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05g}
O=gpurun_out/$TAG
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
P="timeout -k 10 300 python tools/dropin_probe.py 65536 6"
MPCEKF_BOUNCE_MAX=0 $P > $O/dropin_probe_direct.jsonl 2> $O/dropin_probe_direct.err || exit 1
$P > $O/dropin_probe_bounce.jsonl 2> $O/dropin_probe_bounce.err || exit 1
D="timeout -k 10 300 python tools/dropin_bench.py --route capi"
$D --cells 65536 --steps 20 > $O/dropin_capi_65536.json 2> $O/dropin_capi_65536.err || exit 1
$D --cells 1024 --steps 40 > $O/dropin_capi_1024.json 2> $O/dropin_capi_1024.err || exit 1
timeout -k 10 300 python tools/dropin_bench.py --route device --cells 65536 --steps 20 > $O/dropin_mex_65536.json \
  2> $O/dropin_mex_65536.err || exit 1
B="timeout -k 10 300 python bench.py --no-cpu"
for n in 1024 4096 16384; do
  $B --cells-per-gpu $n > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
done
