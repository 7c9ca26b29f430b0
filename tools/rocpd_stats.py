#!/usr/bin/env python3
"""Per-kernel count / mean / total duration from a rocprofv3 results.db (sqlite).

    python tools/rocpd_stats.py gpurun_out/X/run_results.db [name-substring]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = db.execute("select name, count(*), avg(duration), sum(duration) from kernels group by name "
                  "order by sum(duration) desc").fetchall()
tot = sum(r[3] for r in rows)
for name, cnt, avg, s in rows:
    short = re.sub(r"\(\(anonymous namespace\)::", "", re.sub(r"\((const )?mk::.*", "", name))
    if flt in name:
        print(f"{cnt:8d} {avg / 1e3:10.3f} us {s / 1e6:10.2f} ms {100 * s / tot:6.2f}%  {short[:110]}")
