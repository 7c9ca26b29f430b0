#!/usr/bin/env python3
"""Why the C-ABI stage route's mpc call can stall: the drop-in sequence (plant -> ekf ->
linearize -> lin_fields -> mpc_diag -> mpc) at 65,536 cells with lin_fields' result
handled four ways, timing each stage's host call.

  free    : the [n, 14] result dropped at once (the drop-ins' pattern)
  keep    : every result kept alive until the end
  reuse   : one preallocated result array filled every step (out=)
  skip    : no lin_fields call

Usage: python tools/dropin_probe.py [cells] [steps]"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

P = importlib.import_module("mpc-ekf4fastcharge_amd")
M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
SLOTS = np.array(list(range(20, 27)) + [28] + list(range(29, 35)), dtype=np.int32)


def run(mode, n, steps, rom, soc0, tc):
    tim = {}
    kept = []
    with M.Context(rom, n, M.make_config(bounds=True)) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)
        buf = np.empty((n, SLOTS.size))
        for k in range(steps + 2):
            t = {}

            def timed(name, f, *a, **kw):
                t0 = time.perf_counter()
                r = f(*a, **kw)
                t[name] = time.perf_counter() - t0
                return r

            v = timed("plant", ctx.OB_step, uk, tc)
            zk, _, _ = timed("ekf", ctx.iterEKF, v, uk, tc, xind=False)
            timed("linearize", ctx.EKFmatsHandler, None, None, tc, keep=True)
            if mode == "free":
                timed("lin_fields", ctx.lin_fields, SLOTS)
            elif mode == "keep":
                kept.append(timed("lin_fields", ctx.lin_fields, SLOTS))
            elif mode == "reuse":
                timed("lin_fields", ctx.lin_fields, SLOTS, out=buf)
            timed("mpcdiag", ctx.mpc_diag, None)
            uk, _, _ = timed("mpc", ctx.iterMPC, None, zk[:, -1], cost=True)
            if k >= 2:
                for key, val in t.items():
                    tim[key] = tim.get(key, 0.0) + val
    return {key: round(val / steps * 1e3, 3) for key, val in tim.items()}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rom = P.make_synth_rom(lookup="quintic")
    soc0, tc = bench.batch_inputs(n)
    for mode in ("free", "keep", "reuse", "skip", "free"):
        print(json.dumps({"mode": mode, "cells": n, "ms_per_stage": run(mode, n, steps, rom, soc0, tc)}), flush=True)


if __name__ == "__main__":
    main()
