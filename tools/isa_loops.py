#!/usr/bin/env python3
"""Per-loop instruction mix of one kernel in a hipcc -S listing.

    python tools/isa_loops.py listing.s KERNEL_SYMBOL_PREFIX"""
import re
import sys

text = open(sys.argv[1]).read()
start = text.index("\n" + sys.argv[2])
L = text[start:text.index("s_endpgm", start)].split("\n")
PATS = {"VALU": r"\s+v_", "f64": r"\s+v_\w*f64", "SALU": r"\s+s_", "LDS": r"\s+ds_", "VMEM": r"\s+(global|buffer)_",
        "scratch": r"\s+scratch_", "accv": r"\s+v_accvgpr"}
lab = {}
for i, l in enumerate(L):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        lab[m.group(1)] = i
for i, l in enumerate(L):
    m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(1) in lab and lab[m.group(1)] < i:
        body = L[lab[m.group(1)]:i + 1]
        mix = " ".join(f"{k} {sum(1 for x in body if re.match(p, x))}" for k, p in PATS.items())
        print(f"loop {m.group(1)} lines {lab[m.group(1)]}-{i}: {mix}")
print("whole kernel:", " ".join(f"{k} {sum(1 for x in L if re.match(p, x))}" for k, p in PATS.items()))
