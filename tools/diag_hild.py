#!/usr/bin/env python3
"""Per-step k_hild time vs Hildreth sweep statistics (mean / per-wave max)."""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
P = importlib.import_module("mpc-ekf4fastcharge_amd")
rom = P.make_synth_rom()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1010
soc0, tc = bench.batch_inputs(n)
ctx = M.Context(rom, n, M.make_config(bounds=True))
ctx.init_cells(soc0, tc)
ctx.set_timing(True)
rows = []
for k in range(steps):
    ctx.get_timing()
    out = ctx.step(1, outputs=("nexec",))
    t = ctx.get_timing()
    ne = out["nexec"][0]
    wmax = ne.reshape(-1, 64).max(1)
    rows.append(dict(k=k, hild_ms=t["hild"][0], cell_ms=t["cell"][0], flush_ms=t["flush"][0],
                     mean=float(ne.mean()), wmax=float(wmax.mean()), frac100=float((ne == 100).mean())))
json.dump(rows, open(sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/diag_hild.json", "w"))
a = np.array([[r["hild_ms"], r["mean"], r["wmax"]] for r in rows])
# least squares: hild_ms ~ c0 + c1 * wmax
A = np.c_[np.ones(len(a)), a[:, 2]]
coef = np.linalg.lstsq(A, a[:, 0], rcond=None)[0]
print("mean hild ms %.4f  mean nexec %.2f  mean wave-max %.2f  fit: %.4f ms + %.5f ms/sweep" %
      (a[:, 0].mean(), a[:, 1].mean(), a[:, 2].mean(), coef[0], coef[1]))
for r in rows[::100]:
    print(r)
