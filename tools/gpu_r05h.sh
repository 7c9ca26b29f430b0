#!/bin/bash
# Round-5 pass h: same-box A/B of the branch-free v3 lookup (libmpcekf_bf.so, MPCEKF_PL_BRANCHFREE=1)
# against the default library at configs[2], twice interleaved; the drop-in probe with only copies up
# to 4 MiB bounced.
#   gpurun --timeout 900 -- 'bash tools/gpu_r05h.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05h}
O=gpurun_out/$TAG
mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu"
V=mpc-ekf4fastcharge_amd/_build/libmpcekf_bf.so
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
MPCEKF_LIB=$V timeout -k 10 600 $T tests/test_gpu_handles.py tests/test_gpu_horizons.py > $O/bf_tests.log 2>&1 || exit 1
for rep in 1 2; do
  $B > $O/bench_main_$rep.json 2> $O/bench_main_$rep.err || exit 1
  MPCEKF_LIB=$V $B > $O/bench_bf_$rep.json 2> $O/bench_bf_$rep.err || exit 1
done
MPCEKF_BOUNCE_MAX=4194304 timeout -k 10 300 python tools/dropin_probe.py 65536 6 > $O/dropin_probe_4m.jsonl \
  2> $O/dropin_probe_4m.err || exit 1
