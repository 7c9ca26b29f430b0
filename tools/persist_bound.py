#!/usr/bin/env python3
"""How much a persistent multi-step kernel could save on the Hildreth term (VERDICT r02
"do this" 6): per-step kernels pay, every step, the sweeps of the slowest cell of the
whole grid (a grid-wide barrier per step: sum over steps of the global maximum); a
kernel in which each wave advances its own 64 cells through the steps pays, per wave,
the sum over steps of that wave's maximum, and finishes with its slowest wave.

    python tools/persist_bound.py [ncells] [steps]   (C oracle, CPU; bench.py's inputs)

Prints the two sums over bench.py's timed window (steps 10..10+steps) and their ratio,
the bound on the Hildreth part of a persistent kernel's gain."""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import oracle_c  # noqa: E402

P = importlib.import_module("mpc-ekf4fastcharge_amd")

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
rom = P.make_synth_rom()
soc0, tc = bench.batch_inputs(n)
out = oracle_c.run(rom, soc0, tc, 10 + steps, nthreads=os.cpu_count() or 1)
ne = out["nexec"][10:].astype(np.int64)                 # [steps, n]
glob = int(ne.max(axis=1).sum())                        # per-step kernels: sum of global maxima
w = ne[:, : n - n % 64].reshape(steps, -1, 64).max(axis=2)  # [steps, waves]
per_wave = w.sum(axis=0)
# regrouping cells into waves by their mean sweep count (a persistent kernel could bin)
order = np.argsort(-ne.mean(axis=0), kind="stable")
ws = ne[:, order[: n - n % 64]].reshape(steps, -1, 64).max(axis=2).sum(axis=0)
res = {"cells": n, "steps": steps, "window": [10, 10 + steps],
       "sum_global_max_sweeps": glob,
       "persistent_max_over_waves_of_sum_wave_max": int(per_wave.max()),
       "persistent_mean_over_waves": float(per_wave.mean()),
       "ratio_persistent_vs_per_step": float(per_wave.max() / glob),
       "binned_by_mean_sweeps_max_over_waves": int(ws.max()),
       "ratio_binned_vs_per_step": float(ws.max() / glob),
       "mean_sweeps_per_cell_step": float(ne.mean()),
       "steps_with_a_maxIter_cell": int((ne.max(axis=1) >= 100).sum())}
print(json.dumps(res, indent=1))
