#!/usr/bin/env python3
"""Benchmark: batched MPC+EKF control steps/s on MI355X (BASELINE.json metric).

One step = one closed-loop pass of runMPC.m:84-111 (OB_step -> iterEKF ->
EKFmatsHandler -> iterMPC/hildreth) over every cell of the batch.  Workload:
65 536 cells per GPU (BASELINE.json configs[2], the north_star target config),
synthetic NMC30-like ROM (3 x 21 set-points), Np=5 / Nc=2, SOC0 ~ U[5,30] %,
TC ~ U[20,30] degC (seed 0x5EED).  Multi-GPU: one process per GPU, cells sharded
contiguously with no collective on the data path (weak scaling); the only
collectives are the timing barrier and the max-over-ranks of the elapsed time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cells-per-gpu C]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)

METRIC = "MPC+EKF control steps/sec (whole batch), Np=5 Nc=2; 1/2/4/8 MI355X"


def algorithmic_bytes_per_cell(NM, ncon, bounds, lazy_h=32, Np=5, Nc=2):
    """Algorithmic HBM bytes each kernel moves per cell per launch:
    the state it must read and write once, with nothing re-read.

    flush: the all-model time update, run as k_flush every lazy_h steps: every EKF
           record (xhat 5 + packed Sigma 15) and plant state (6) read + written,
           the model timestamps (2 x NM int32) read + written, the two input rings.
    cell : the 4 corner EKF records read + written, their timestamps, the step's
           ring input, per-cell scalars/constants, outputs u/v/soc/phise, zk,
           the QP record (+ the 14-double boundzk hand-off record).
    bounds: the hand-off record and corner 1's packed Sigma read, 4 per-cell
           constants read, boundzk (28) written.
    plant: the 4 corner plant states read + written, timestamps, ring writes,
           per-cell scalars.
    hild : the QP record read, lambda read + written, outputs.
    """
    flush = 2 * 8 * NM * (20 + 6) + 2 * 2 * 4 * NM + 2 * 8 * lazy_h
    zk = 8 * 28
    cell = 4 * 2 * 8 * 20 + 4 * 2 * 4 + 8 + 20 * 8 + 4 * 8 + zk + 51 * 8 + (14 * 8 if bounds else 0)
    plant = 4 * 2 * 6 * 8 + 4 * 2 * 4 + 2 * 8 + 12 * 8 + 8
    hild = 51 * 8 + 2 * 8 * ncon + 4 * 8
    if (Np, Nc) != (5, 2):
        # wide horizons (mpcekf_wide.hip): k_cell hands over the 35-double linearisation
        # record + zk(end); the QP record E, F, Hv, He, Hs, gamma, e, Ru, uk_1 and the
        # hildreth.m setup X (ncon x Nc), K, H_ii are written by k_mpc_wide and read back
        prob = Nc * Nc + Nc + 4 * Np + ncon + 2
        cell = cell - 51 * 8 + 36 * 8
        hild = 2 * 8 * (36 + prob + ncon * (Nc + 2)) + 2 * 8 * ncon + 4 * 8
    out = dict(flush=flush, cell=cell, plant=plant, hild=hild)
    if bounds:
        out["bounds"] = 14 * 8 + 15 * 8 + 4 * 8 + 28 * 8
    return out


def survey_bytes_per_cell_step(NM, ncon):
    """the whole step's persistent state read + written once."""
    return 416 * NM + 16 * ncon + 160


FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (AMD spec; FMA = 2 flops); no FMA here -> 39.3 reachable


def batch_inputs(n, seed=0x5EED):
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(5, 30, n), rng.uniform(20, 30, n)


def cpu_baseline(rom, soc0, tc, cells, steps, threads, Np=5, Nc=2):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    t0 = time.perf_counter()
    oracle_c.run(rom, soc0[:cells], tc[:cells], steps, nthreads=threads, Np=Np, Nc=Nc)
    dt = time.perf_counter() - t0
    return dict(value=cells * steps / dt, unit="cell-steps/s", cores=threads, kind="port",
                sample=f"C oracle (oracle/mpcekf_oracle.c, -O3 fp64, OpenMP) on the first {cells} cells "
                       f"of the workload x {steps} steps from init, {threads} host threads, {dt:.1f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cells-per-gpu", type=int, default=65536)
    ap.add_argument("--bounds", type=int, default=1, help="compute boundzk every step (iterEKF.m:186-205)")
    ap.add_argument("--np", type=int, default=5, help="prediction horizon (configs[4]: 20)")
    ap.add_argument("--nc", type=int, default=2, help="control horizon (configs[4]: 10)")
    ap.add_argument("--cpu-cells", type=int, default=32768)
    ap.add_argument("--cpu-steps", type=int, default=0, help="default: warmup + steps (the GPU run's steps)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing-every", type=int, default=8,
                    help="per-kernel HIP-event timing on every N-th step of the timed region (N | 32)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
    rom = P.make_synth_rom()
    cpg = args.cells_per_gpu
    total = cpg * world
    soc0_all, tc_all = batch_inputs(total)
    sl = slice(rank * cpg, (rank + 1) * cpg)
    cfg = M.make_config(bounds=bool(args.bounds), Np=args.np, Nc=args.nc)
    ncon = 4 * args.nc + 3 * args.np
    ctx = M.Context(rom, cpg, cfg, device=local)
    ctx.init_cells(soc0_all[sl], tc_all[sl])
    dev = torch.device("cuda", local)
    K, W = args.steps, args.warmup
    outs = [torch.empty((max(K, W), cpg), dtype=torch.float64, device=dev) for _ in range(4)]
    nex = torch.empty((max(K, W), cpg), dtype=torch.int32, device=dev)
    ptrs = [t.data_ptr() for t in outs] + [nex.data_ptr()]
    if W:
        ctx.step_device(W, *ptrs)
    ctx.set_timing(args.timing_every)
    ctx.get_timing()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ctx.step_device(K, *ptrs)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    tim = ctx.get_timing()
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    status = ctx.get_state()["status"]
    nerr = int((status & 1).sum())
    u_last = outs[0][K - 1].double().cpu().numpy() if K else np.zeros(0)
    mean_nexec = float(nex[:K].float().mean().item()) if K else 0.0
    ctx.close()

    if rank == 0:
        cell_steps = total * K
        value = cell_steps / dt if dt > 0 else 0.0
        bpc = algorithmic_bytes_per_cell(rom.NM, ncon, bool(args.bounds), Np=args.np, Nc=args.nc)
        # HIP-event averages over the sampled launches (--timing-every); every flush step is
        # sampled, so a kernel's share of a step is its average x its launches per step
        n_flush = K // 32 + (1 if K % 32 else 0)
        per_kernel = {k: dict(ms_per_launch=tim[k][0] / max(tim[k][1], 1), launches_timed=tim[k][1],
                              launches=(n_flush if k == "flush" else K))
                      for k in tim if tim[k][1] > 0}
        for v in per_kernel.values():
            v["ms_total"] = v["ms_per_launch"] * v["launches"]
        # the dominant kernel = the largest share of the timed region (k_flush runs every 32 steps)
        dom = max(per_kernel, key=lambda k: per_kernel[k]["ms_total"])
        ms = per_kernel[dom]["ms_per_launch"]
        achieved = bpc[dom] * cpg / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        pmc = {}
        if os.path.exists(args.pmc):
            try:
                pmc = json.load(open(args.pmc))
            except Exception:
                pmc = {}
        traffic = pmc.get("per_launch_bytes", {}).get(dom)
        flops = pmc.get("fp64_flops_per_launch", {}).get(dom)
        fp64 = None
        if flops and ms > 0:
            tf = flops / (ms * 1e-3) / 1e12
            fp64 = {"achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                    "flops_per_launch": flops, "source": os.path.relpath(args.pmc, ROOT)}
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(rom, soc0_all, tc_all, min(args.cpu_cells, cpg), args.cpu_steps or (W + K),
                               args.cpu_threads, Np=args.np, Nc=args.nc)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "cell-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": dt / K * 1e3 if K else 0.0,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (synthetic NMC30-like ROM; SOC0~U[5,30]%, TC~U[20,30]C, seed 0x5EED)",
            "config": {
                "workload": f"{cpg} cells per GPU ({total} total), Np={args.np} Nc={args.nc}, closed loop runMPC.m:84-111 "
                            f"incl. plant, boundzk={'on' if args.bounds else 'off'}",
                "cells_per_gpu": cpg, "total_cells": total, "Np": args.np, "Nc": args.nc, "models_per_cell": rom.NM,
                "rom_outputs": rom.nz, "parallelism": f"cell-shard x{world} (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "algorithmic_bytes_per_cell": bpc[dom],
                "fp64": fp64,
                "step_equivalent": {
                    "bytes_per_cell_step": survey_bytes_per_cell_step(rom.NM, ncon),
                    "achieved": value * survey_bytes_per_cell_step(rom.NM, ncon) / 1e9, "unit": "GB/s",
                    "note": "SURVEY.md 8(d): whole-step state r+w per cell-step x cell-steps/s",
                },
            },
            "kernels": {k: dict(ms_per_launch=round(v["ms_per_launch"], 5), launches=v["launches"],
                                launches_timed=v["launches_timed"],
                                ms_per_step=round(v["ms_total"] / K, 5) if K else None,
                                gbs_algorithmic=round(bpc[k] * cpg / (v["ms_per_launch"] * 1e-3) / 1e9, 1)
                                if v["ms_per_launch"] > 0 else None)
                        for k, v in per_kernel.items()},
            "cpu_baseline": cpu,
            "checks": {"cells_in_error": nerr, "mean_nexec": round(mean_nexec, 3),
                       "u_last_mean": float(np.nanmean(u_last)) if u_last.size else None},
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
