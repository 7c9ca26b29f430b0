#!/usr/bin/env python3
"""Throughput of the route north_star prescribes for MATLAB hosts: runMPC.m's loop body
(runMPC.m:85-103) as the stage calls the drop-ins in matlab/dropin/*.m issue through the
MEX gateway (matlab/mpcekf_mex.c), driven here without MATLAB through the MEX API test
shim (tests/mexshim.py).  One step, per the drop-ins:

  OB_step.m        mpcekf_mex('scalars', h, [1 2])        SOCnAvg/SOCpAvg (OB_step.m:226-228)
                   mpcekf_mex('plant', h, uk, Tc)          OB_step.m:1
  iterEKF.m        mpcekf_mex('ekf', h, v, uk, Tk)          iterEKF.m:30
                   mpcekf_mex('scalars', h, [3 4 5])        ekfData.x0 / SigmaX0 / priorI, warn, status
  EKFmatsHandler.m mpcekf_mex('linearize', h, zk, xm, xg, Tk)  EKFmatsHandler.m:1
  iterMPC.m        mpcekf_mex('mpcdiag', h, lin, [])        iterMPC.m:53-60 (poles / sv)
                   mpcekf_mex('mpc', h, lin, zk(end, :))    iterMPC.m:1,89-95

It reports cell-steps/s and the host<->device bytes per cell-step, split into the
stage calls' own arguments/results (what the reference's function signatures pass) and
the per-step state reads the drop-ins add ('scalars'; round 3 used a whole get_state
here, ~13 KB per cell twice a step).  The fused mpcekf_step is bench.py's figure.

    python tools/dropin_bench.py --cells 65536 --steps 40 --warmup 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-diag", action="store_true", help="skip the mpcdiag call (poles / sv)")
    a = ap.parse_args()
    import importlib

    import mexshim
    import bench
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    rom = P.make_synth_rom()
    n = a.cells
    soc0, tc = bench.batch_inputs(n)
    nbytes = {"args": 0, "state": 0}

    def mex(kind, cmd, *args, nargout=1):
        out = mexshim.mex(cmd, *args, nargout=nargout)
        outs = out if isinstance(out, tuple) else (out,)
        nbytes[kind] += sum(x.nbytes for x in args if isinstance(x, np.ndarray) and x.dtype != np.uint64)
        nbytes[kind] += sum(np.asarray(x).nbytes for x in outs if x is not None)
        return out

    h = mexshim.mex("create", mexshim.rom_struct(rom), {"flags": 1.0}, 0.0, float(n))
    try:
        mexshim.mex("init", h, soc0, tc, nargout=0)
        uk = np.zeros((1, n))
        tk = tc[None, :].copy()

        def step():
            nonlocal uk
            s = mex("state", "scalars", h, np.array([[1.0, 2.0]]))
            v = mex("args", "plant", h, uk, tk)
            zk, zbk, xm, xg = mex("args", "ekf", h, v, uk, tk, nargout=4)
            s, warn, status = mex("state", "scalars", h, np.array([[3.0, 4.0, 5.0]]), nargout=3)
            lin = mex("args", "linearize", h, zk, xm, xg, tk)
            if not a.no_diag:
                mex("args", "mpcdiag", h, lin, np.zeros((0, 0)), nargout=2)
            out = mex("args", "mpc", h, lin, zk[-1:, :], nargout=6)
            uk = out[0]
            return out

        for _ in range(a.warmup):
            step()
        nbytes.update(args=0, state=0)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = step()
        dt = time.perf_counter() - t0
        u_last = out[0]
    finally:
        mexshim.mex("destroy", h, nargout=0)
    # the fused path on the same cells and steps, for the bits
    ref = M.runMPC(rom, soc0, tc, a.warmup + a.steps)["u"][-1]
    same = bool(np.array_equal(u_last.ravel(), ref))
    line = {
        "what": "MATLAB drop-in stage route (matlab/dropin/*.m command sequence) through the MEX gateway, "
                "driven by the MEX API test shim (no MATLAB); host arrays in and out every call",
        "cells": n, "steps": a.steps, "warmup": a.warmup, "mpcdiag": not a.no_diag,
        "cell_steps_per_s": n * a.steps / dt, "ms_per_step": dt / a.steps * 1e3,
        "host_bytes_per_cell_step": {k: v / (n * a.steps) for k, v in nbytes.items()},
        "u_last_equals_fused": same,
        "build_id": M._lib.load().mpcekf_build_id().decode(),
    }
    print(json.dumps(line), flush=True)
    if not same:
        sys.exit("dropin_bench: the stage route's u differs from the fused step")


if __name__ == "__main__":
    main()
