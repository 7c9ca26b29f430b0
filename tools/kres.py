#!/usr/bin/env python3
"""Per-kernel resource usage from a device assembly file (hipcc --cuda-device-only -S):
VGPRs, AGPRs, SGPRs, scratch bytes, spill counts and instruction counts, for the kernels
whose (mangled) name matches a filter.  Usage: python tools/kres.py file.s [substr ...]"""
import re
import sys


def kernels(text):
    out = {}
    for m in re.finditer(r"\n(_Z\S+):[^\n]*\n.*?\n\s*s_endpgm", text, re.S):
        name = m.group(1)
        body = m.group(0)
        ninst = sum(1 for ln in body.split("\n") if re.match(r"\s+[sv]_|\s+ds_|\s+global_|\s+buffer_|\s+flat_|\s+scratch_", ln))
        out[name] = {"inst": ninst, "scratch_ops": body.count("scratch_"), "agpr_moves": body.count("v_accvgpr")}
    meta = {}
    for blk in re.findall(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.S):
        name, b = blk
        g = lambda k: int(re.search(rf"\.amdhsa_{k}\s+(\d+)", b).group(1)) if re.search(rf"\.amdhsa_{k}\s+(\d+)", b) else None
        meta[name] = {"vgpr": g("next_free_vgpr"), "sgpr": g("next_free_sgpr"), "scratch": g("private_segment_fixed_size"),
                      "acc_offset": g("accum_offset")}
    for n in out:
        out[n].update(meta.get(n, {}))
    return out


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    flt = sys.argv[2:]
    for n, v in sorted(kernels(text).items()):
        if all(f in n for f in flt):
            print(n[:90], v)
