#!/usr/bin/env python3
"""Experiment: one batch split into G contexts (own HIP stream each) stepped from G host
threads at once, against one context over the whole batch.  Each group's kernels run at one
wave per SIMD on part of the chip; if the groups drift out of phase, one group's record
read/write bursts (k_cell, k_flush) overlap another's issue-bound Hildreth sweeps.

    python tools/stream_split.py --cells 65536 --groups 1 2 4 --steps 1000 --warmup 10
"""
import argparse
import importlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(P, M, rom, soc0, tc, G, K, W, Np, Nc):
    import torch
    n = len(soc0)
    cfg = M.make_config(bounds=True, Np=Np, Nc=Nc)
    bounds = [(g * n // G, (g + 1) * n // G) for g in range(G)]
    ctxs, bufs = [], []
    dev = torch.device("cuda", 0)
    for lo, hi in bounds:
        c = M.Context(rom, hi - lo, cfg, device=0)
        c.init_cells(soc0[lo:hi], tc[lo:hi])
        o = [torch.empty((max(K, W), hi - lo), dtype=torch.float64, device=dev) for _ in range(4)]
        o.append(torch.empty((max(K, W), hi - lo), dtype=torch.int32, device=dev))
        ctxs.append(c)
        bufs.append(o)

    def go(i, k):
        c, o = ctxs[i], bufs[i]
        c.step_device(k, *[t.data_ptr() for t in o])

    def all_groups(k):
        th = [threading.Thread(target=go, args=(i, k)) for i in range(G)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    all_groups(W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    all_groups(K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    u = np.concatenate([o[0][K - 1].cpu().numpy() for o in bufs])
    for c in ctxs:
        c.close()
    return dt, u


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=65536)
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--np", type=int, default=5)
    ap.add_argument("--nc", type=int, default=2)
    a = ap.parse_args()
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    bench = importlib.import_module("bench")
    rom = P.make_synth_rom()
    soc0, tc = bench.batch_inputs(a.cells)
    ref = None
    for G in a.groups:
        dt, u = run(P, M, rom, soc0, tc, G, a.steps, a.warmup, a.np, a.nc)
        same = None if ref is None else bool(np.array_equal(u.view(np.int64), ref.view(np.int64)))
        if ref is None:
            ref = u
        print(json.dumps(dict(groups=G, cells=a.cells, steps=a.steps, ms_per_step=dt / a.steps * 1e3,
                              cell_steps_per_s=a.cells * a.steps / dt, u_last_bitwise_vs_first=same)), flush=True)


if __name__ == "__main__":
    main()
