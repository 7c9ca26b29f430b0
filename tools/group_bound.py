#!/usr/bin/env python3
"""Bound for a two-group schedule of the fused step: every flush window
(32 steps) the cells whose Hildreth took >= THETA sweeps in the previous window form
the "slow" group, the rest the "fast" group; each group runs its own per-step kernel
chain on its own stream for the window (cells are independent), and the groups join
at the flush.  Step cost model from the round-3 measurements at 65,536 cells
(profiles/r03j_bench.json, r03j_bench_1024.json): a group's non-Hildreth chain (plant +
cell + bounds) is BIG_US for the large group and SMALL_US for a group of at most a few
thousand cells; k_hild costs H0_US + H1_US x (the group's slowest cell's sweeps).

    python tools/group_bound.py [ncells] [theta ...]

Prints the modelled time of the window loop against the single-group baseline."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BIG_US, SMALL_US = 41 + 103 + 25, 26 + 75 + 20   # plant + cell + bounds
H0_US, H1_US = 24.0, 1.3                         # k_hild: fixed + per sweep of the slowest cell
FLUSH_US = 486.0                                 # k_flush per 32-step window
W = 32

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
thetas = [int(t) for t in sys.argv[2:]] or [10, 20, 40]
cache = f"/tmp/nexec_{n}.npy"
if os.path.exists(cache):
    ne = np.load(cache)
else:
    import importlib
    import bench
    from oracle import oracle_c
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    soc0, tc = bench.batch_inputs(n)
    ne = oracle_c.run(P.make_synth_rom(), soc0, tc, 1010, nthreads=os.cpu_count() or 1)["nexec"].astype(np.int32)
    np.save(cache, ne)
ne = ne[10:1010]                                  # bench.py's window
steps = ne.shape[0]
base = sum(BIG_US + H0_US + H1_US * ne[k].max() for k in range(steps)) + FLUSH_US * steps / W
res = {"cells": n, "steps": steps, "model_us": {"big_chain": BIG_US, "small_chain": SMALL_US, "hild": [H0_US, H1_US]},
       "baseline_ms": base / 1e3, "groups": {}}
for th in thetas:
    tot, nslow = 0.0, []
    prev = np.zeros(n, bool)
    for w0 in range(0, steps, W):
        blk = ne[w0:w0 + W]
        slow = prev
        fast = ~slow
        tf = sum(BIG_US + H0_US + H1_US * (blk[k][fast].max() if fast.any() else 0) for k in range(blk.shape[0]))
        ts = sum(SMALL_US + H0_US + H1_US * blk[k][slow].max() for k in range(blk.shape[0])) if slow.any() else 0.0
        tot += max(tf, ts) + FLUSH_US
        nslow.append(int(slow.sum()))
        prev = blk.max(axis=0) >= th
    res["groups"][th] = {"modelled_ms": tot / 1e3, "speedup": base / tot, "slow_cells_mean": float(np.mean(nslow)),
                         "slow_cells_max": int(np.max(nslow))}
print(json.dumps(res, indent=1))
