"""Diagnostic: GPU vs C oracle at Np=20/Nc=10 for the near-limit cells; per-cell first
divergence step.  Writes gpurun_out/diag_wide.npz."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_c  # noqa: E402

P = importlib.import_module("mpc-ekf4fastcharge_amd")
M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
rom = P.make_synth_rom()
soc0 = np.array([93.0, 94.0, 94.5, 95.0, 96.0, 90.0, 10.0, 50.0])
tc = np.array([25.0, 20.0, 30.0, 25.0, 25.0, 22.0, 25.0, 28.0])
steps = 300
ref = oracle_c.run(rom, soc0, tc, steps, nthreads=8, Np=20, Nc=10)
out = M.runMPC(rom, soc0, tc, steps, cfg=M.make_config(Np=20, Nc=10))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "diag_wide.npz"), **{"g_" + k: v for k, v in out.items()},
         **{"r_" + k: v for k, v in ref.items()})
for c in range(len(soc0)):
    d = np.abs(out["u"][:, c] - ref["u"][:, c])
    first = np.argmax(d > 0) if (d > 0).any() else -1
    ne = np.argmax(out["nexec"][:, c] != ref["nexec"][:, c]) if (out["nexec"][:, c] != ref["nexec"][:, c]).any() else -1
    dv = np.abs(out["v"][:, c] - ref["v"][:, c])
    fv = np.argmax(dv > 0) if (dv > 0).any() else -1
    print(f"cell {c} soc0 {soc0[c]}: first u diff step {first}, first v diff {fv}, first nexec diff {ne}, "
          f"max |du| {d.max():.3e}, nexec==100 frac {(ref['nexec'][:, c] == 100).mean():.2f}")
