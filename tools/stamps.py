#!/usr/bin/env python3
"""Where k_cell's time goes: per-section shader cycles (profiling build).

    python mpc-ekf4fastcharge_amd/build.py --stamps
    MPCEKF_LIB=mpc-ekf4fastcharge_amd/_build/libmpcekf_stamps.so python tools/stamps.py [ncells] [steps] [lookup]

lookup: the ROM's electrode tables (rom.make_synth_rom: "linear" v2 tables, "quintic" /
"cubic" v3 polynomials; default linear, the round-4 figures).

Runs the bench workload; after each step k in a sample it reads the stamps and
reports the median over waves of each section's cycles (max over the wave's
lanes at each boundary, i.e. the wave's critical path)."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
P = importlib.import_module("mpc-ekf4fastcharge_amd")
NAMES = ["plant (simStep) + scalar loads + lockout", "get_xind1", "catch-up1", "get_vars1", "chatV+gains", "meas_update x4",
         "get_xind2 + catch-up2", "get_vars2", "boundzk record", "mats_handler", "mpc_setup"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
lookup = sys.argv[3] if len(sys.argv) > 3 else "linear"
rom = P.make_synth_rom(lookup=lookup)
soc0, tc = bench.batch_inputs(n)
ctx = M.Context(rom, n, M.make_config(bounds=True))
ctx.init_cells(soc0, tc)
acc = []
pacc = []
PNAMES = ["entry: blob staging + barrier", "scalar loads + bracket + two_nearest", "corner gather issue + Cdleff/res0/SOC", "corner replay",
          "rows + blend (DPP)", "clamps, k0, asinh, Uocp, Rf, V", "stores + corner advance"]
for k in range(steps):
    ctx.step(1, outputs=())
    if k % 25 == 5:
        st = ctx.get_stamps()
        if st is None:
            sys.exit("not a profiling build: set MPCEKF_LIB to _build/libmpcekf_stamps.so")
        w = st.reshape(st.shape[0], -1, 64).max(axis=2).astype(np.float64)  # [stamp][64 cells]
        d = np.diff(w[:12], axis=0)                                         # [section][wave]
        acc.append(np.median(d, axis=1))
        dp = np.diff(np.concatenate([w[19:20], w[12:19]]), axis=0)  # k_plant(4): entry, sections
        pacc.append(np.median(dp, axis=1))
a = np.array(acc)
tot = a.sum(1)
print(f"k_cell sections ({lookup} tables; median over waves, shader cycles; {len(a)} sampled steps, total median {np.median(tot):.0f}):")
for i, nm in enumerate(NAMES):
    print(f"  {nm:44s} {np.median(a[:, i]):9.0f}  ({100 * np.median(a[:, i] / tot):4.1f} %)")
p = np.array(pacc)
ptot = p.sum(1)
if not np.any(ptot):
    sys.exit(0)  # the plant ran inside k_cell (its first section): no k_plant launch to report
print(f"k_plant sections (median, shader cycles; total median {np.median(ptot):.0f}):")
for i, nm in enumerate(PNAMES):
    print(f"  {nm:40s} {np.median(p[:, i]):9.0f}  ({100 * np.median(p[:, i] / ptot):4.1f} %)")
