#!/usr/bin/env python3
"""Table-vs-handle gap of the electrode lookups (DESIGN.md §3, round-4 review item 1).

Runs the numpy oracle (oracle/oracle_np.py, MATLAB-faithful) with the synthetic ROM's
closed-form ``cellData.function`` handles called at every reference call site
(``cfg["handles"]``), and with the same handles tabulated: the v2 linear tables
(201 / 101 theta points) and the v3 Hermite cubics with the exact Arrhenius factor at
several theta resolutions.  Reports, per output (u, v, soc, phise), the largest relative
difference from the handle run over the steps where the handle run is well-conditioned
(tests/envelope.py's per-step ulp envelope is the reference for which steps that is;
here the whole trajectory up to ``--upto``) and the first step where 1e-6 is exceeded.

    python tools/handle_gap.py [--steps 3001] [--cells runmpc|batch8] [--out profiles/r05_handle_gap.json]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_np as O  # noqa: E402

P = importlib.import_module("mpc-ekf4fastcharge_amd")
KEYS = ("u", "v", "soc", "phise")


def cells(which):
    if which == "runmpc":
        return np.array([10.0]), np.array([25.0])
    rng = np.random.Generator(np.random.PCG64(0x5EED))
    return rng.uniform(5, 30, 8), rng.uniform(20, 30, 8)


def run(rom, soc0, tc, steps, handles):
    outs = [O.run_cell(rom, s, t, steps, {"handles": handles}) for s, t in zip(soc0, tc)]
    return {k: np.stack([o[k] for o in outs], axis=1) for k in KEYS + ("nexec",)}


def gap(ref, out, tol=1e-6):
    res = {}
    for k in KEYS:
        a, b = ref[k], out[k]
        rel = np.abs(b - a) / np.maximum(np.abs(a), 1e-300)
        rel = np.where(np.isnan(a) & np.isnan(b), 0.0, rel)
        worst = np.nanmax(rel, axis=1)
        bad = np.nonzero(worst > tol)[0]
        res[k] = {"max_rel": float(np.nanmax(worst)), "first_step_over_1e-6": int(bad[0]) if bad.size else None,
                  "median_rel": float(np.nanmedian(worst))}
    res["nexec_equal_steps"] = int((ref["nexec"] == out["nexec"]).all(axis=1).sum())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3001)
    ap.add_argument("--cells", default="runmpc")
    ap.add_argument("--ntab", default="257,513,1025")
    ap.add_argument("--lookups", default="cubic,quintic")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    soc0, tc = cells(a.cells)
    t0 = time.time()
    base = P.make_synth_rom()
    ref = run(base, soc0, tc, a.steps, True)
    rep = {"cells": a.cells, "steps": a.steps, "handle_run_s": round(time.time() - t0, 1), "variants": {}}
    for name, rom in [("v2 linear 201", base), ("v2 linear 101", P.make_synth_rom(ntab=101))] + \
            [(f"v3 {lk} {n}", P.make_synth_rom(lookup=lk, ntab=n)) for lk in a.lookups.split(",") for n in map(int, a.ntab.split(","))]:
        g = gap(ref, run(rom, soc0, tc, a.steps, False))
        rep["variants"][name] = g
        print(name, json.dumps({k: g[k] for k in KEYS}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
