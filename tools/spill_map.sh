#!/bin/bash
# Where a kernel spills: device ISA with line info (-g), scratch stores / AGPR writes
# counted per source line.  Usage: bash tools/spill_map.sh mpcekf_kernels.hip SYMBOL_PREFIX [-Dextra...]
SRC=$1; SYM=$2; shift 2
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -g -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=200000 \
  -DMPCEKF_SRC_HASH='"x"' "$@" --cuda-device-only -S mpc-ekf4fastcharge_amd/csrc/$SRC -o /tmp/spill_$$.s 2>/dev/null
python3 - /tmp/spill_$$.s "$SYM" <<'PY'
import re, sys, collections
text = open(sys.argv[1]).read()
st = text.index("\n" + sys.argv[2])
L = text[st:text.index("s_endpgm", st)].split("\n")
files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
         for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', text)}
cur = None
c = {k: collections.Counter() for k in ("scratch_store", "scratch_load", "v_accvgpr_write", "v_accvgpr_read")}
for l in L:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    for k in c:
        if k in l:
            c[k][cur] += 1
for k, cnt in c.items():
    print(f"{k}: total {sum(cnt.values())}; " + ", ".join(f"{f}:{n} x{v}" for (f, n), v in cnt.most_common(12)))
PY
rm -f /tmp/spill_$$.s
