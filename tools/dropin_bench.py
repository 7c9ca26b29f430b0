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
    ap.add_argument("--route", default="device",
                    choices=("device", "host", "capi", "capi-async", "c", "c-async", "c-reuse", "c-async-reuse"),
                    help="device: the drop-ins' round-5 sequence (zk / Xind / lin stay on the device, 14 "
                         "doubles of lin read back); host: the round-4 sequence (every array through the "
                         "host); capi: the device sequence through ctypes (mpcekf.py) instead of the MEX "
                         "gateway, so the shim's marshalling is separated out; capi-async: the same with the "
                         "_async stage twins, Vcell handed to iterEKF on the device, one synchronisation per "
                         "step (iterMPC); c / c-async: the capi sequences driven from C "
                         "(tools/dropin_loop.c: fresh malloc'ed outputs every call, as mxArrays), so the "
                         "Python binding's per-call work is separated out as well; -reuse: output arrays "
                         "allocated once, so the caller's allocator is separated out too")
    ap.add_argument("--rom-lookup", default="quintic", choices=("linear", "cubic", "quintic"))
    a = ap.parse_args()
    if a.route in ("capi", "capi-async"):
        return capi(a)
    if a.route.startswith("c-") or a.route == "c":
        return c_loop(a)
    import importlib

    import mexshim
    import bench
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    rom = P.make_synth_rom(lookup=a.rom_lookup)
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

        e = np.zeros((0, 0))
        lin_slots = np.array([list(range(21, 28)) + [29] + list(range(30, 36))], dtype=float)

        def step():
            nonlocal uk
            s = mex("state", "scalars", h, np.array([[1.0, 2.0]]))
            v = mex("args", "plant", h, uk, tk)
            if a.route == "host":
                zk, zbk, xm, xg = mex("args", "ekf", h, v, uk, tk, nargout=4)
            else:  # Xind crosses back too (the drop-in keeps MPC.iT / iZ from it), zk / Xind are not sent back
                zk, zbk, xm, xg = mex("args", "ekf", h, v, uk, tk, nargout=4)
            s, warn, status = mex("state", "scalars", h, np.array([[3.0, 4.0, 5.0]]), nargout=3)
            if a.route == "host":
                lin = mex("args", "linearize", h, zk, xm, xg, tk)
            else:
                mex("args", "linearize", h, e, e, e, tk)
                mex("args", "linfields", h, lin_slots)     # Cphi, Dphi, bphi, xhat (runMPC.m:95-96)
                lin = e
            if not a.no_diag:
                mex("args", "mpcdiag", h, lin, e, nargout=2)
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
        "route": a.route, "rom_lookup": a.rom_lookup,
        "cells": n, "steps": a.steps, "warmup": a.warmup, "mpcdiag": not a.no_diag,
        "cell_steps_per_s": n * a.steps / dt, "ms_per_step": dt / a.steps * 1e3,
        "host_bytes_per_cell_step": {k: v / (n * a.steps) for k, v in nbytes.items()},
        "u_last_equals_fused": same,
        "build_id": M._lib.load().mpcekf_build_id().decode(),
    }
    print(json.dumps(line), flush=True)
    if not same:
        sys.exit("dropin_bench: the stage route's u differs from the fused step")


def capi(a):
    """The drop-ins' device-route stage sequence through the C-ABI directly (ctypes, host
    buffers, mpcekf.py), timed per stage, bytes counted from the arrays each call moves."""
    import importlib

    import bench
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    rom = P.make_synth_rom(lookup=a.rom_lookup)
    n = a.cells
    soc0, tc = bench.batch_inputs(n)
    slots = np.array(list(range(20, 27)) + [28] + list(range(29, 35)), dtype=np.int32)
    tim = {k: 0.0 for k in ("scalars", "plant", "ekf", "linearize", "lin_fields", "mpcdiag", "mpc")}
    nb = {k: 0 for k in tim}
    asy = a.route == "capi-async"
    with M.Context(rom, n, M.make_config(bounds=True)) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)

        def timed(k, f, *args, **kw):
            t0 = time.perf_counter()
            r = f(*args, **kw)
            tim[k] += time.perf_counter() - t0
            return r

        def step(count):
            nonlocal uk
            ctx.asynchronous = asy
            timed("scalars", ctx.get_scalars, ("SOCnAvg", "SOCpAvg"))          # OB_step.m:226-228
            v = timed("plant", ctx.OB_step, uk, tc)
            # async: Vcell reaches iterEKF on the device (vk = None), its host copy at the sync
            zk, zb, xi = timed("ekf", ctx.iterEKF, None if asy else v, uk, tc)
            timed("scalars", ctx.get_scalars, ("x0", "SigmaX0", "priorI"), flags=True)   # ekfData fields
            timed("linearize", ctx.EKFmatsHandler, None, None, tc, keep=True)
            f = timed("lin_fields", ctx.lin_fields, slots)
            if not a.no_diag:
                timed("mpcdiag", ctx.mpc_diag, None)
            ctx.asynchronous = False   # iterMPC synchronises: every earlier output is written
            # async: SOCk_1 = zk(end) from the device zk (runMPC.m:99), the host zk not yet written
            uk, ne, cost = timed("mpc", ctx.iterMPC, None, None if asy else zk[:, -1], cost=True)
            if count:
                nb["scalars"] += (16 + 24 + 8) * n
                nb["plant"] += 3 * 8 * n
                nb["ekf"] += 3 * 8 * n + zk.nbytes + zb.nbytes + xi["model"].nbytes + xi["gamma"].nbytes
                nb["linearize"] += 8 * n
                nb["lin_fields"] += f.nbytes
                nb["mpcdiag"] += 0 if a.no_diag else (14 + 7) * 8 * n
                nb["mpc"] += 8 * n + uk.nbytes + ne.nbytes + sum(np.asarray(x).nbytes for x in cost.values()
                                                                  if np.asarray(x).dtype != object)
            return uk

        for _ in range(a.warmup):
            step(False)
        for k in tim:
            tim[k] = 0.0
        t0 = time.perf_counter()
        for _ in range(a.steps):
            u_last = step(True)
        dt = time.perf_counter() - t0
    ref = M.runMPC(rom, soc0, tc, a.warmup + a.steps)["u"][-1]
    same = bool(np.array_equal(u_last, ref))
    line = {"what": "the drop-ins' device-route stage sequence through the C-ABI (ctypes, host buffers): "
                    "plant -> ekf -> linearize (kept on device) -> lin_fields (14 doubles) -> mpc_diag -> mpc",
            "route": a.route, "rom_lookup": a.rom_lookup, "cells": n, "steps": a.steps, "warmup": a.warmup,
            "copy_threads": os.environ.get("MPCEKF_COPY_THREADS", "default"),
            "chunk": os.environ.get("MPCEKF_CHUNK", "default"),
            "mpcdiag": not a.no_diag, "cell_steps_per_s": n * a.steps / dt, "ms_per_step": dt / a.steps * 1e3,
            "ms_per_step_by_stage": {k: v / a.steps * 1e3 for k, v in tim.items()},
            "host_bytes_per_cell_step": {k: v / (n * a.steps) for k, v in nb.items()},
            "host_bytes_per_cell_step_total": sum(nb.values()) / (n * a.steps),
            "u_last_equals_fused": same, "build_id": M._lib.load().mpcekf_build_id().decode()}
    print(json.dumps(line), flush=True)
    if not same:
        sys.exit("dropin_bench: the C-ABI stage route's u differs from the fused step")


def c_loop(a):
    """The capi stage sequence driven from C (tools/dropin_loop.c) on a context made here."""
    import ctypes as C
    import importlib
    import subprocess

    import bench
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    bdir = os.path.join(ROOT, "mpc-ekf4fastcharge_amd", "_build")
    so = os.path.join(bdir, "libdropin_loop.so")
    src = os.path.join(ROOT, "tools", "dropin_loop.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-std=c11", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "include"), src,
                        "-L" + bdir, "-lmpcekf", "-Wl,-rpath,$ORIGIN", "-o", so], check=True)
    lib = C.CDLL(so)
    rom = P.make_synth_rom(lookup=a.rom_lookup)
    n = a.cells
    soc0, tc = bench.batch_inputs(n)
    sc = M.Context.SCALARS
    sa = np.array([sc.index(k) for k in ("SOCnAvg", "SOCpAvg")], dtype=np.int32)
    sb = np.array([sc.index(k) for k in ("x0", "SigmaX0", "priorI")], dtype=np.int32)
    fields = np.array(list(range(20, 27)) + [28] + list(range(29, 35)), dtype=np.int32)
    uk = np.zeros(n)
    ms = np.zeros(7)
    tot, byt = C.c_double(), C.c_double()
    ip = lambda x: x.ctypes.data_as(C.POINTER(C.c_int32))
    dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))
    with M.Context(rom, n, M.make_config(bounds=True)) as ctx:
        ctx.init_cells(soc0, tc)
        lib.dropin_loop.restype = C.c_int
        rc = lib.dropin_loop(ctx.h, C.c_int64(n), C.c_int32(ctx.nz), C.c_int32(a.steps),
                             C.c_int32(a.warmup), C.c_int32(("async" in a.route) + 2 * ("reuse" in a.route)), dp(tc), ip(sa), len(sa), ip(sb),
                             len(sb), ip(fields), len(fields), dp(uk), dp(ms), C.byref(tot), C.byref(byt))
        if rc:
            sys.exit(f"dropin_loop failed: {rc} {M._lib.load().mpcekf_last_error().decode()}")
    ref = M.runMPC(rom, soc0, tc, a.warmup + a.steps)["u"][-1]
    same = bool(np.array_equal(uk, ref))
    names = ("scalars", "plant", "ekf", "linearize", "lin_fields", "mpcdiag", "mpc")
    line = {"what": "the drop-ins' device-route stage sequence through the C-ABI, driven from C (tools/dropin_loop.c, "
                    + ("host output arrays allocated once" if "reuse" in a.route else
                       "fresh malloc'ed host outputs every call") +
                    "): plant -> ekf -> linearize (kept on device) -> lin_fields (14 doubles) -> mpc_diag -> mpc",
            "route": a.route, "rom_lookup": a.rom_lookup, "cells": n, "steps": a.steps, "warmup": a.warmup,
            "copy_threads": os.environ.get("MPCEKF_COPY_THREADS", "default"),
            "chunk": os.environ.get("MPCEKF_CHUNK", "default"), "mpcdiag": True,
            "cell_steps_per_s": n * a.steps / (tot.value * 1e-3), "ms_per_step": tot.value / a.steps,
            "ms_per_step_by_stage": {k: float(ms[i]) / a.steps for i, k in enumerate(names)},
            "host_bytes_per_cell_step_total": byt.value,
            "u_last_equals_fused": same, "build_id": M._lib.load().mpcekf_build_id().decode()}
    print(json.dumps(line), flush=True)
    if not same:
        sys.exit("dropin_bench: the C-driven stage route's u differs from the fused step")


if __name__ == "__main__":
    main()
