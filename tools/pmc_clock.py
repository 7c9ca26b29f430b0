#!/usr/bin/env python3
"""Effective shader clock per kernel from a rocprofv3 --pmc pass that holds SQ_BUSY_CYCLES:
the counter summed over the 32 shader engines, divided by 32 and by the dispatch's own
duration (Start/End_Timestamp of the same CSV row).  Usage: pmc_clock.py PASS_DIR"""
import csv
import glob
import re
import sys
from collections import defaultdict

import numpy as np

acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "SQ_BUSY_CYCLES":
            continue
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        if not m:
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        if dur > 0:
            acc[m.group(1)].append((float(r["Counter_Value"]) / 32 / dur / 1e9, dur * 1e3))
for k, v in sorted(acc.items(), key=lambda kv: -np.median([x[1] for x in kv[1]])):
    a = np.array(v)
    print(f"{k:28s} n={len(v):5d}  clock GHz median {np.median(a[:, 0]):.2f} (p10 {np.percentile(a[:, 0], 10):.2f}, "
          f"p90 {np.percentile(a[:, 0], 90):.2f})  duration ms median {np.median(a[:, 1]):.3f}")
