#!/bin/bash
# Register / scratch / occupancy of the kernels in one source (device-only compile with
# the library's flags).  Usage: bash tools/kru.sh mpcekf_kernels.hip [name-regex] [-Dextra...]
SRC=$1; shift
PAT=${1:-.}; shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=200000 \
  -DMPCEKF_SRC_HASH='"x"' "$@" --cuda-device-only -c mpc-ekf4fastcharge_amd/csrc/$SRC -o /tmp/kru_$$.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import re, sys
pat = re.compile(sys.argv[1]); cur = None; out = {}
for l in sys.stdin:
    m = re.search(r'Function Name: (\S+)', l)
    if m: cur = m.group(1); out[cur] = {}; continue
    m = re.search(r'remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill): (\d+)', l)
    if m and cur: out[cur][m.group(1).split(' [')[0].replace(' ', '_')] = int(m.group(2))
for k, v in out.items():
    if pat.search(k): print(f'{k[:70]:70s} ' + ' '.join(f'{a}={b}' for a, b in v.items()))
" "$PAT"
rm -f /tmp/kru_$$.o
