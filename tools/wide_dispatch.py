#!/usr/bin/env python3
"""k_hild_wide per dispatch: duration over the bench window (kernel trace, rocpd db) and,
from a --pmc pass holding SQ_WAVES / SQ_INSTS_VALU / SQ_WAVE_CYCLES / SQ_BUSY_CYCLES, the
VALU instructions and wave cycles per wave and the effective clock of chosen dispatches.

    python tools/wide_dispatch.py TRACE_DB PMC_PASS_DIR > out.json"""
import csv
import glob
import json
import sqlite3
import sys
from collections import defaultdict

import numpy as np

db = sqlite3.connect(sys.argv[1])
d = np.array([r[1] for r in db.execute("select name, duration from kernels order by start")
              if "k_hild_wide<" in r[0]], float) / 1e6
out = {"trace_ms_per_50_dispatches": [round(float(d[i:i + 50].mean()), 3) for i in range(0, len(d), 50)],
       "trace_mean_ms": float(d.mean()), "trace_median_ms": float(np.median(d))}
per = defaultdict(dict)
for f in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_hild_wide<" in r["Kernel_Name"]:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            per[int(r["Dispatch_Id"])]["ms"] = dur
ks = sorted(per)
rows = []
for i in (5, 100, 300, 400, 500, 550, 600):
    if i < len(ks):
        p = per[ks[i]]
        rows.append({"dispatch": i, "ms": round(p["ms"], 3), "valu_per_wave": round(p["SQ_INSTS_VALU"] / p["SQ_WAVES"]),
                     "wave_cycles": round(4 * p["SQ_WAVE_CYCLES"] / p["SQ_WAVES"]),
                     "cycles_per_valu_per_wave": round(4 * p["SQ_WAVE_CYCLES"] / p["SQ_INSTS_VALU"], 2),
                     "clock_GHz": round(p["SQ_BUSY_CYCLES"] / 32 / (p["ms"] * 1e-3) / 1e9, 2)})
out["pmc_dispatches"] = rows
print(json.dumps(out, indent=1))
