#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc CSV directories to per-kernel averages of every counter.

Usage: pmc_sq.py OUT_JSON DIR [DIR ...]   (each DIR one counter pass, e.g. pmc_probe.sh's a..e)
Output: {"build_id": ..., "per_kernel": {kernel: {counter: mean per dispatch}}, "derived": {...}}
Derived per kernel (when the counters are present): VALU instructions per wave, the
fraction of wave-cycles a wave spent waiting on anything / on LDS, LDS bank-conflict
cycles per LDS instruction.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(kn):
    kn = kn.replace("(anonymous namespace)::", "").split("(")[0]
    kn = kn.replace("void ", "").replace("mk::", "")
    return kn.strip()


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    acc[short(row.get("Kernel_Name", ""))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    per = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    der = {}
    for k, c in per.items():
        d = {}
        if c.get("SQ_WAVES"):
            if "SQ_INSTS_VALU" in c:
                d["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
            if "SQ_INSTS_LDS" in c:
                d["lds_insts_per_wave"] = c["SQ_INSTS_LDS"] / c["SQ_WAVES"]
        if c.get("SQ_WAVE_CYCLES"):
            for nm in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                       "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if nm in c:
                    d[nm.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = c[nm] / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
            d["lds_bank_conflict_cycles_per_lds_inst"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"]
        if c.get("SQ_BUSY_CYCLES") and "SQ_INSTS_VALU" in c:
            d["valu_insts_per_busy_cycle"] = c["SQ_INSTS_VALU"] / c["SQ_BUSY_CYCLES"]
        der[k] = d
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pmc_traffic import bench_build_id
    bid = None
    for d in dirs:
        bid = bid or bench_build_id(os.path.dirname(d.rstrip("/")) or ".")
    res = {"build_id": bid, "passes": dirs, "per_kernel": per, "derived": der,
           "note": "rocprofv3 counters per dispatch, averaged over dispatches; SQ_* cycle counters are "
                   "summed over SEs/XCDs by rocprofv3, so only ratios of them are meaningful"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
