#!/usr/bin/env python3
"""Per-call cost of the fused step as a control loop drives it (mpcekf_step with
nsteps = 1 every period, outputs on the device): direct launches vs hipGraph replay
(mpcekf_set_graph).  Prints one JSON line per (cells, mode).

    python tools/graph_bench.py [--cells 1024 65536] [--calls 400]"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, nargs="+", default=[1024, 65536])
    ap.add_argument("--calls", type=int, default=400)
    a = ap.parse_args()
    import torch
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    rom = P.make_synth_rom()
    for n in a.cells:
        rng = np.random.Generator(np.random.PCG64(0x5EED))
        soc0, tc = rng.uniform(5, 30, n), rng.uniform(20, 30, n)
        outs = [torch.empty((1, n), dtype=torch.float64, device="cuda:0") for _ in range(4)]
        nex = torch.empty((1, n), dtype=torch.int32, device="cuda:0")
        ptrs = [o.data_ptr() for o in outs] + [nex.data_ptr()]
        res = {}
        for mode in ("launches", "graph"):
            with M.Context(rom, n) as ctx:
                ctx.init_cells(soc0, tc)
                ctx.set_graph(mode == "graph")
                for _ in range(20):  # warm-up (and the capture)
                    ctx.step_device(1, *ptrs)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.calls):
                    ctx.step_device(1, *ptrs)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / a.calls
                res[mode] = dt
                u = outs[0].cpu().numpy().copy()
            res[mode + "_u"] = u
        same = bool(np.array_equal(res["launches_u"], res["graph_u"]))
        for mode in ("launches", "graph"):
            print(json.dumps({"cells": n, "mode": mode, "calls": a.calls, "ms_per_call": res[mode] * 1e3,
                              "cell_steps_per_s": n / res[mode], "u_bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()
