#!/usr/bin/env python3
"""Reduce rocprofv3 PMC CSVs to per-launch HBM bytes for each bench kernel.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
exactly half the bytes of a wide (16 B/lane) coalesced streaming read
(MI355X_MICROARCH.md §HBM), so reads are doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  Output: JSON with per_launch_bytes{plant,flush,cell,hild,bounds} (flush = the all-model
time update of the fused path) and fp64_flops_per_launch.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# kernel (exact name prefix) -> bench stage; a stage's per-step figure is the sum of
# its kernels' per-dispatch averages (each launches once per step)
KERNELS = {"k_plant(": "plant", "k_plant4<": "plant", "k_flush(": "flush", "k_cell<": "cell", "k_hild(": "hild", "k_hild_slow(": "hild",
           "k_bounds<": "bounds", "k_bulk(": "bulk",
           # wide horizons (mpcekf_wide.hip): bench.py's "cell" slot times k_cell + k_mpc_wide,
           # its "hild" slot the whole hildreth.m pipeline (prep, binning, sweeps, exact path, finish)
           "k_mpc_wide<": "cell", "k_hild_prep<": "hild", "k_hild_bin<": "hild", "k_hild_sort(": "hild",
           "k_hild_wide<": "hild", "k_hild_wide_slow<": "hild", "k_mpc_wide_finish<": "hild"}


def bench_build_id(base):
    """The build id the profiled bench printed (its JSON line's checks.build_id): the
    library that ran on the box, which the local tree may since have changed."""
    for path in sorted(glob.glob(os.path.join(base, "*.log")) + glob.glob(os.path.join(base, "*.json"))):
        try:
            with open(path) as f:
                for line in f:
                    if line.startswith("{") and '"build_id"' in line:
                        return json.loads(line)["checks"]["build_id"]
        except (OSError, ValueError, KeyError):
            continue
    return None


def read_counter(d, name, by_kernel=False):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != name:
                    continue
                kn = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
                for k in KERNELS:
                    if ("mk::" + k) in kn or (" " + k) in kn or kn.startswith(k):
                        vals[k].append(float(row["Counter_Value"]))
    if by_kernel:
        return {k.rstrip("(<"): sum(v) / len(v) for k, v in vals.items() if v}
    stage = defaultdict(float)
    for k, v in vals.items():
        if v:
            stage[KERNELS[k]] += sum(v) / len(v)
    return dict(stage)


def main():
    import argparse
    import importlib
    ap = argparse.ArgumentParser()
    ap.add_argument("base")
    ap.add_argument("--cells", type=int, default=65536)
    ap.add_argument("--np", type=int, default=5)
    ap.add_argument("--bounds", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--rom-lookup", default="quintic", help="when the bench line does not say (bench.py default)")
    a = ap.parse_args()
    base = a.base
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    bid = bench_build_id(base)
    if bid is None:
        bid = importlib.import_module("mpc-ekf4fastcharge_amd._lib").load().mpcekf_build_id().decode()
    fetch = read_counter(os.path.join(base, "fetch"), "FETCH_SIZE")
    write = read_counter(os.path.join(base, "write"), "WRITE_SIZE")
    # the electrode tables the profiled bench ran (its JSON line's config.rom_lookup; bench.py
    # attaches these figures only to a run with the same tables)
    lookup = a.rom_lookup
    for root, _, files in os.walk(base):
        for fn in files:
            if fn.endswith((".json", ".log")):
                try:
                    with open(os.path.join(root, fn)) as f:
                        for line in f:
                            if line.startswith("{") and '"rom_lookup"' in line:
                                lookup = json.loads(line)["config"].get("rom_lookup", lookup)
                except (OSError, ValueError, KeyError):
                    pass
    out = {"unit": "bytes per launch", "build_id": bid, "cells": a.cells, "Np": a.np, "rom_lookup": lookup,
           "bounds": a.bounds, "steps": a.steps, "fetch_kib_raw": fetch, "write_kib_raw": write,
           "correction": "reads x2 (gfx950 FETCH_SIZE halves 16-B/lane streaming reads)",
           "per_launch_bytes": {}}
    for k in set(fetch) | set(write):
        out["per_launch_bytes"][k] = 2 * fetch.get(k, 0.0) * 1024 + write.get(k, 0.0) * 1024
    # the same per kernel (a stage's figure is the sum of its kernels')
    fk = read_counter(os.path.join(base, "fetch"), "FETCH_SIZE", by_kernel=True)
    wk = read_counter(os.path.join(base, "write"), "WRITE_SIZE", by_kernel=True)
    out["per_kernel_bytes"] = {k: 2 * fk.get(k, 0.0) * 1024 + wk.get(k, 0.0) * 1024 for k in set(fk) | set(wk)}
    # FP64 work per launch: the SQ_INSTS_VALU_*_F64 counters count wave instructions;
    # x64 lanes (an upper bound when EXEC is partial), FMA = 2 flops
    fd = os.path.join(base, "fp64")
    if os.path.isdir(fd):
        cnt = {nm: read_counter(fd, f"SQ_INSTS_VALU_{nm}_F64") for nm in ("ADD", "MUL", "FMA", "TRANS")}
        out["fp64_flops_per_launch"] = {
            k: 64.0 * (cnt["ADD"].get(k, 0) + cnt["MUL"].get(k, 0) + cnt["TRANS"].get(k, 0) + 2 * cnt["FMA"].get(k, 0))
            for k in set().union(*[set(v) for v in cnt.values()])}
        out["fp64_wave_instructions_per_launch"] = cnt
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
