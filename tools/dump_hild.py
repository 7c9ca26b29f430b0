#!/usr/bin/env python3
"""Dumps the real k_hild inputs of one fused step of the bench workload for
offline replay by tools/micro/hild_micro (--state):
    python tools/dump_hild.py STEP OUT.bin [ncells]
Layout: int64 n, then prob [51][n], lambda-in [23][n] (field-major), hflag int32 [n]."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
P = importlib.import_module("mpc-ekf4fastcharge_amd")
step, out = int(sys.argv[1]), sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
rom = P.make_synth_rom()
soc0, tc = bench.batch_inputs(n)
ctx = M.Context(rom, n, M.make_config(bounds=True))
ctx.init_cells(soc0, tc)
ctx.step(step, outputs=())
lam = ctx.get_state()["lam"]          # [n][23], the warm start k_hild reads
o = ctx.step(1, outputs=("nexec",))
prob, hflag = ctx.get_hild_problems()
with open(out, "wb") as f:
    np.array([n], dtype=np.int64).tofile(f)
    prob.astype(np.float64).tofile(f)
    np.ascontiguousarray(lam.T).astype(np.float64).tofile(f)
    hflag.astype(np.int32).tofile(f)
ne = o["nexec"][0]
np.save(out + ".nexec.npy", ne)
print(f"step {step}: {int(hflag.sum())} QPs, nexec mean {ne.mean():.2f} max {ne.max()}, "
      f"waves at 100: {(ne.reshape(-1, 64).max(1) == 100).sum()}")
