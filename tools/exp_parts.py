"""Experiment: the 65,536-cell batch as P concurrent sub-batch contexts (one HIP stream
each, driven from P host threads; ctypes releases the GIL) against one context.
Prints cell-steps/s for P = 1, 2, 4."""
import importlib
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

P = importlib.import_module("mpc-ekf4fastcharge_amd")
M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
rom = P.make_synth_rom()
N, K, W = 65536, int(os.environ.get("STEPS", "1000")), 10
rng = np.random.Generator(np.random.PCG64(0x5EED))
soc0, tc = rng.uniform(5, 30, N), rng.uniform(20, 30, N)
cfg = M.make_config(bounds=True)
dev = torch.device("cuda", 0)
for parts in (1, 2, 4, 1):
    n = N // parts
    ctxs, bufs = [], []
    for p in range(parts):
        c = M.Context(rom, n, cfg)
        c.init_cells(soc0[p * n:(p + 1) * n], tc[p * n:(p + 1) * n])
        outs = [torch.empty((K, n), dtype=torch.float64, device=dev) for _ in range(4)]
        nex = torch.empty((K, n), dtype=torch.int32, device=dev)
        ctxs.append(c)
        bufs.append([t.data_ptr() for t in outs] + [nex.data_ptr()])
        bufs[-1].append((outs, nex))
    for c, b in zip(ctxs, bufs):
        c.step_device(W, *b[:5])
    torch.cuda.synchronize()
    ths = [threading.Thread(target=c.step_device, args=(K, *b[:5])) for c, b in zip(ctxs, bufs)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"parts {parts}: {N * K / dt:.4e} cell-steps/s, {dt / K * 1e3:.4f} ms/step", flush=True)
    for c in ctxs:
        c.close()
