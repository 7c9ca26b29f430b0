#!/usr/bin/env python3
"""Benchmark: batched MPC+EKF control steps/s on MI355X (BASELINE.json metric).

One step = one closed-loop pass of runMPC.m:84-111 (OB_step -> iterEKF ->
EKFmatsHandler -> iterMPC/hildreth) over every cell of the batch.  Workload:
65 536 cells per GPU (BASELINE.json configs[2], the north_star target config),
synthetic NMC30-like ROM (3 x 21 set-points), Np=5 / Nc=2, SOC0 ~ U[5,30] %,
TC ~ U[20,30] degC (seed 0x5EED).  Multi-GPU: one process per GPU, cells sharded
contiguously with no collective on the data path (weak scaling); the only
collectives are the timing barrier and the max-over-ranks of the elapsed time, run
over gloo by a coordinator child of each rank (the rank process loads one HIP
runtime, libmpcekf's, and never imports torch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cells-per-gpu C | --total-cells T]

--gpus N without torchrun starts N rank processes itself (one per GPU, before any
GPU call); under torchrun the ranks come from RANK/WORLD_SIZE.  configs[3] is
``--gpus 8 --total-cells 1048576`` (131 072 cells per GPU, strong scaling).
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


LAZY_H = 64  # the library's input-ring length = flush period (mpcekf_kernels.hpp MPCEKF_LAZY_H)


def algorithmic_bytes_per_cell(NM, ncon, bounds, lazy_h=LAZY_H, Np=5, Nc=2, bounds_kernel=True, plant_kernel=False,
                               hild_kernel=True):
    """Algorithmic HBM bytes each kernel moves per cell per launch:
    the state it must read and write once, with nothing re-read.

    flush: the all-model time update, run as k_flush every lazy_h steps: every EKF
           record (xhat 5 + packed Sigma 15) and plant state (6) read + written,
           the model timestamps (2 x NM int32) read + written, the two input rings.
    cell : the 4 corner EKF records read + written, their timestamps, the step's
           ring input, per-cell scalars/constants, outputs u/v/soc/phise, zk,
           the QP record (+ the 14-double boundzk hand-off record).
    bounds: (k_bounds, the library default: MPCEKF_CELL_BOUNDS=0) the hand-off record and
           corner 1's packed Sigma read, 4 per-cell constants read, boundzk (28) written;
           with bounds_kernel=False k_cell evaluates boundzk itself (corner 1's Sigma
           read, boundzk written, no record).
    plant: the 4 corner plant states read + written, timestamps, ring writes,
           per-cell scalars (k_cell's own bytes when it runs the plant, the default).
    hild : the QP record read, lambda read + written, outputs.
    """
    flush = 2 * 8 * NM * (20 + 6) + 2 * 2 * 4 * NM + 2 * 8 * lazy_h
    zk = 8 * 28
    cell = 4 * 2 * 8 * 20 + 4 * 2 * 4 + 8 + 20 * 8 + 4 * 8 + zk + 51 * 8 + (14 * 8 if bounds else 0)
    plant = 4 * 2 * 6 * 8 + 4 * 2 * 4 + 2 * 8 + 12 * 8 + 8
    hild = 51 * 8 + 2 * 8 * ncon + 4 * 8
    if (Np, Nc) != (5, 2):
        # wide horizons (mpcekf_wide.hip): k_cell hands over the 35-double linearisation
        # record + zk(end); the QP record E, F, Hv, He, Hs, gamma, e, Ru, uk_1 is written by
        # k_mpc_wide and read back; k_hild_prep hands k_hild_wide chol(E) (Nc(Nc+1)/2) and K
        # (ncon), and k_hild_wide forms X and H_ii itself (MPCEKF_WIDE_XPRO, the default)
        prob = Nc * Nc + Nc + 4 * Np + ncon + 2
        cell = cell - 51 * 8 + 36 * 8
        hild = 2 * 8 * (36 + prob + Nc * (Nc + 1) // 2 + ncon) + 2 * 8 * ncon + 4 * 8
    out = dict(flush=flush, cell=cell, plant=plant, hild=hild)
    if not plant_kernel:  # k_cell runs OB_step's simStep first (KRom::cell_plant): its bytes are k_cell's
        out["cell"] = cell = cell + plant
        del out["plant"]
    if not hild_kernel:  # hildreth.m at the end of k_cell (Np = 5 fused step): its bytes are k_cell's
        out["cell"] = cell = cell + hild
        del out["hild"]
    if bounds and bounds_kernel:
        out["bounds"] = 14 * 8 + 15 * 8 + 4 * 8 + 28 * 8
    elif bounds:  # k_cell evaluates boundzk: no hand-off record; corner 1's Sigma read, boundzk written
        out["cell"] = cell - 14 * 8 + 15 * 8 + 28 * 8
    return out


def survey_bytes_per_cell_step(NM, ncon):
    """the whole step's persistent state read + written once."""
    return 416 * NM + 16 * ncon + 160


FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (AMD spec; FMA = 2 flops); no FMA here -> 39.3 reachable


def batch_inputs(n, seed=0x5EED):
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(5, 30, n), rng.uniform(20, 30, n)


def rom_grid(args):
    """make_synth_rom set-point grid: NM = temps x socs (default 3 x 21 = 63); T in
    [15, 35] degC and SOC in [0, 100] % evenly."""
    kw = {}
    if args.rom_temps:
        kw["T_degC"] = tuple(np.linspace(15.0, 35.0, args.rom_temps)) if args.rom_temps > 1 else (25.0,)
    if args.rom_socs:
        kw["SOC_pct"] = tuple(np.linspace(0.0, 100.0, args.rom_socs))
    kw["lookup"] = getattr(args, "rom_lookup", "linear")
    return kw


def shard_range(total, world, rank):
    """Contiguous cell range [start, stop) of one rank (runMPC.m:83-112 has no cross-cell
    term, so any split gives the same bits per cell)."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def cpu_threads_default():
    """The host cores this process may use: the affinity mask, capped by OMP_NUM_THREADS
    (the GPU box sets it to its 16-CPU share; os.cpu_count() there is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_baseline(rom, soc0, tc, cells, steps, threads, Np=5, Nc=2):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    t0 = time.perf_counter()
    oracle_c.run(rom, soc0[:cells], tc[:cells], steps, nthreads=threads, Np=Np, Nc=Nc)
    dt = time.perf_counter() - t0
    # configs[0]: the runMPC.m cell (SOC0 10 %, 25 degC), the whole 3001-step charge on one core
    t1 = time.perf_counter()
    oracle_c.run(rom, np.array([10.0]), np.array([25.0]), 3001, nthreads=1, Np=Np, Nc=Nc)
    d1 = time.perf_counter() - t1
    return dict(value=cells * steps / dt, unit="cell-steps/s", cores=threads, kind="port",
                host_cpus=os.cpu_count(),
                sample=f"C oracle (oracle/mpcekf_oracle.c, -O3 fp64, OpenMP) on the first {cells} cells "
                       f"of the workload x {steps} steps from init, {threads} host threads of {os.cpu_count()} "
                       f"logical CPUs, {dt:.1f} s",
                configs0={"cells": 1, "steps": 3001, "cores": 1, "wall_s": d1, "steps_per_s": 3001 / d1,
                          "what": "runMPC.m cell (SOC0 10 %, 25 degC), full charge, 1 thread"})


def count_gpus(sysfs="/sys/class/kfd/kfd/topology/nodes", dev="/dev/dri", env=None):
    """GPUs this process could open, counted without any HIP / HSA call and without torch:
    the KFD topology nodes with SIMDs (GPU agents) whose render node /dev/dri/renderD<minor>
    is accessible, then limited by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES (the runtime applies them in that order).  The rank launcher's
    parent uses it so that it never maps a GPU runtime before it spawns the ranks."""
    env = os.environ if env is None else env
    n = 0
    try:
        nodes = sorted(os.listdir(sysfs), key=lambda x: int(x) if x.isdigit() else 1 << 30)
    except OSError:
        nodes = []
    for nd in nodes:
        props = {}
        try:
            with open(os.path.join(sysfs, nd, "properties")) as f:
                for line in f:
                    kv = line.split()
                    if len(kv) == 2 and kv[1].lstrip("-").isdigit():
                        props[kv[0]] = int(kv[1])
        except OSError:
            continue
        if props.get("simd_count", 0) <= 0:
            continue                                  # a CPU agent
        minor = props.get("drm_render_minor", -1)
        node = os.path.join(dev, f"renderD{minor}")
        if minor >= 0 and os.path.exists(node) and os.access(node, os.R_OK | os.W_OK):
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def _parent_maps_gpu_runtime():
    """Lines of /proc/self/maps naming a GPU runtime (HIP, HSA, torch's bundled ones)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if any(k in ln for k in
                           ("libamdhip64", "libhsa-runtime64", "libtorch_hip", "libtorch_cuda"))})
    except OSError:
        return []


def launch_ranks(args):
    """--gpus N without torchrun: N worker processes, one per GPU, started before this
    process touches the GPU (it counts devices from sysfs, count_gpus, and refuses to
    spawn if a GPU runtime is mapped here); exits with the first failing rank's code."""
    import socket
    import subprocess
    if not (args.dry_run or args.share_device):
        have = count_gpus()
        if have < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible (KFD topology)")
    mapped = _parent_maps_gpu_runtime()
    if os.environ.get("MPCEKF_BENCH_PARENT_MAPS"):   # tests/test_multiproc.py
        with open(os.environ["MPCEKF_BENCH_PARENT_MAPS"], "w") as f:
            f.write("\n".join(mapped))
    if mapped:
        sys.exit(f"bench.py: the rank launcher has a GPU runtime mapped before spawning: {mapped}")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c]
    sys.exit(bad[0] if bad else 0)


class Coordinator:
    """The ranks' timing collectives (barrier, max/sum over ranks) over gloo, run by a
    child process (``bench.py --coordinator``) that this rank starts before it touches the
    GPU.  The rank process itself never imports torch: torch's bundled HIP runtime would
    otherwise be mapped next to the one libmpcekf links (two runtimes in one process, a
    round-3 finding).  The path has no data-path collective (cells are independent,
    SURVEY.md §8(e)); these are the bench contract's barrier and max-over-ranks time."""

    def __init__(self):
        import subprocess
        self.p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--coordinator"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=dict(os.environ))
        self.backend = self._reply()

    def _reply(self):
        line = self.p.stdout.readline()
        if not line:
            code = self.p.wait()
            sys.exit(f"bench.py: timing coordinator exited ({code})")
        return line.strip()

    def _cmd(self, *words):
        self.p.stdin.write(" ".join(str(w) for w in words) + "\n")
        self.p.stdin.flush()
        return self._reply()

    def barrier(self):
        self._cmd("barrier")

    def reduce(self, dt, nerr, nexec_sum):
        """(max over ranks of dt, sum of nerr, sum of nexec_sum)"""
        a, b, c = self._cmd("reduce", repr(float(dt)), repr(float(nerr)), repr(float(nexec_sum))).split()
        return float(a), int(float(b)), float(c)

    def close(self):
        self._cmd("exit")
        self.p.wait(timeout=60)


def coordinator_main():
    """Child of one rank: joins the gloo process group (RANK / WORLD_SIZE / MASTER_* from
    the environment, torchrun's agent store when present) and serves the rank's timing
    collectives over stdin/stdout on CPU tensors."""
    # replies go to a private copy of stdout; anything torch / gloo print goes to stderr
    reply = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    if "RANK" in os.environ:
        dist.init_process_group("gloo")
    else:  # --force-dist outside a launcher: a world of one on a private loopback store
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    print(dist.get_backend(), file=reply, flush=True)
    for line in sys.stdin:
        w = line.split()
        if not w or w[0] == "exit":
            print("bye", file=reply, flush=True)
            break
        if w[0] == "barrier":
            dist.barrier()
            print("ok", file=reply, flush=True)
        elif w[0] == "reduce":
            dt = torch.tensor([float(w[1])], dtype=torch.float64)
            rest = torch.tensor([float(w[2]), float(w[3])], dtype=torch.float64)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            dist.all_reduce(rest, op=dist.ReduceOp.SUM)
            print(repr(float(dt[0])), repr(float(rest[0])), repr(float(rest[1])), file=reply, flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cells-per-gpu", type=int, default=65536, help="weak scaling (default)")
    ap.add_argument("--total-cells", type=int, default=0,
                    help="strong scaling: split this many cells over the ranks (configs[3]: 1048576 on 8)")
    ap.add_argument("--bounds", type=int, default=1, help="compute boundzk every step (iterEKF.m:186-205)")
    ap.add_argument("--np", type=int, default=5, help="prediction horizon (configs[4]: 20)")
    ap.add_argument("--nc", type=int, default=2, help="control horizon (configs[4]: 10)")
    ap.add_argument("--rom-temps", type=int, default=0,
                    help="SURVEY.md 8(d) sensitivity: temperature set-points of the synthetic ROM (default 3)")
    ap.add_argument("--rom-socs", type=int, default=0, help="SOC set-points of the synthetic ROM (default 21)")
    ap.add_argument("--rom-lookup", default="quintic", choices=("linear", "cubic", "quintic"),
                    help="electrode tables (DESIGN.md §3): quintic = ABI v3 theta quintics + Arrhenius "
                         "factor, within 1e-6 of the closed-form handles; linear = the v2 tables")
    ap.add_argument("--cpu-cells", type=int, default=32768)
    ap.add_argument("--cpu-steps", type=int, default=0, help="default: warmup + steps (the GPU run's steps)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="default: the cores this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing-every", type=int, default=8,
                    help="per-kernel HIP-event timing on every N-th step of the timed region (N divides "
                         "the flush period, 64)")
    ap.add_argument("--pmc", default="",
                    help="PMC traffic JSON (tools/pmc_traffic.py); default profiles/pmc_traffic.json, "
                         "profiles/pmc_traffic_np20.json at Np = 20")
    ap.add_argument("--share-device", action="store_true",
                    help="all ranks on device 0 (1-GPU multi-rank test)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: rank/shard/timing orchestration only (CPU tests)")
    ap.add_argument("--force-dist", action="store_true",
                    help="start the timing coordinator (gloo process group) at WORLD_SIZE 1 too")
    ap.add_argument("--coordinator", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.coordinator:
        coordinator_main()
        return
    if not args.pmc:
        args.pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json" if args.np == 5 else f"pmc_traffic_np{args.np}.json")

    period = int(os.environ.get("MPCEKF_FLUSH_PERIOD", str(LAZY_H)))
    if args.timing_every > 1 and period % args.timing_every:
        # report() counts the timed k_flush launches as the region's flushes: every flush
        # step must be a sampled step
        sys.exit(f"bench.py: --timing-every {args.timing_every} must divide the flush period {period}")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    total = args.total_cells or args.cells_per_gpu * world
    lo, hi = shard_range(total, world, rank)
    ncell = hi - lo
    device = 0 if args.share_device else local
    # timing collectives in a gloo child process, started before any GPU call
    coord = Coordinator() if (world > 1 or args.force_dist) else None
    backend = coord.backend if coord else "none"
    print(f"bench.py rank {rank}/{world}: cells [{lo}, {hi}) ({ncell}) on "
          f"{'no device (dry run)' if args.dry_run else f'device {device}'}, process group: {backend}",
          file=sys.stderr, flush=True)
    K, W = args.steps, args.warmup
    runtimes = None

    if args.dry_run:
        # the rank / shard / coordinator path without a GPU (tests/test_multiproc.py): each
        # rank "works" (rank + 1) x 20 ms on its shard, and the reductions carry its cell
        # count and a checksum of its SOC0 so the test can see max-over-ranks timing and
        # shard coverage through the same collectives the GPU run uses
        rom = None
        soc0_all, tc_all = batch_inputs(total)
        if coord:
            coord.barrier()
        t0 = time.perf_counter()
        time.sleep(0.02 * (rank + 1))
        shard_sum = float(soc0_all[lo:hi].sum())
        dt = time.perf_counter() - t0
        tim, nerr, mean_nexec, u_last = {}, ncell, shard_sum / max(ncell, 1), np.zeros(0)
    else:
        P = importlib.import_module("mpc-ekf4fastcharge_amd")
        M = importlib.import_module("mpc-ekf4fastcharge_amd.mpcekf")
        rom = P.make_synth_rom(**rom_grid(args))
        soc0_all, tc_all = batch_inputs(total)
        cfg = M.make_config(bounds=bool(args.bounds), Np=args.np, Nc=args.nc)
        ctx = M.Context(rom, ncell, cfg, device=device)
        ctx.init_cells(soc0_all[lo:hi], tc_all[lo:hi])
        # [steps][cells] trajectories in HBM, allocated by the library's runtime
        rows = max(K, W, 1)
        outs = [M.DeviceBuffer((rows, ncell), np.float64, device) for _ in range(4)]
        nex = M.DeviceBuffer((rows, ncell), np.int32, device)
        if W:
            ctx.step_device(W, *outs, nex)
        ctx.set_timing(args.timing_every)
        ctx.get_timing()
        ctx.sync()
        if coord:
            coord.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        ctx.step_device(K, *outs, nex)
        ctx.sync()
        dt = time.perf_counter() - t0
        tim = ctx.get_timing()
        status = ctx.get_state()["status"]
        nerr = int((status & 1).sum())
        u_last = outs[0].to_host(K)[K - 1] if K else np.zeros(0)
        mean_nexec = float(nex.to_host(K).mean()) if K else 0.0
        build_id = ctx.L.mpcekf_build_id().decode()
        runtimes = M.hip_runtimes()
        for b in outs + [nex]:
            b.free()
        ctx.close()
    if coord:
        # max over ranks of each rank's time from the common barrier to its own sync
        coord.barrier()
        dt, nerr, nexec_sum = coord.reduce(dt, nerr, mean_nexec * ncell)
        mean_nexec = nexec_sum / total
        coord.close()

    if rank == 0:
        cell_steps = total * K
        value = cell_steps / dt if dt > 0 else 0.0
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "cell-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": dt / K * 1e3 if K else 0.0,
            "higher_is_better": True,
            "scaling": "strong" if args.total_cells else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (synthetic NMC30-like ROM; SOC0~U[5,30]%, TC~U[20,30]C, seed 0x5EED)",
            "config": {
                "workload": f"{total} cells ({shard_range(total, world, 0)[1]} on rank 0), Np={args.np} Nc={args.nc}, "
                            f"closed loop runMPC.m:84-111 incl. plant, boundzk={'on' if args.bounds else 'off'}",
                "total_cells": total, "cells_per_gpu": [shard_range(total, world, r)[1] - shard_range(total, world, r)[0]
                                                        for r in range(world)],
                "Np": args.np, "Nc": args.nc, "models_per_cell": rom.NM if rom else None,
                "rom_lookup": args.rom_lookup,
                "rom_outputs": rom.nz if rom else None,
                "parallelism": f"cell-shard x{world} (no data-path collective)",
                "timing_collectives": backend,
                "step_window": [W, W + K], "mean_nexec": round(mean_nexec, 3),
            },
        }
        if args.dry_run:
            line["dry_run"] = True
            line["value"] = None
            # reduced over the ranks: the cells they covered and the sum of their SOC0
            line["dry_run_checks"] = {"cells": nerr, "soc0_sum": mean_nexec * total, "max_dt_s": dt}
            print(json.dumps(line), flush=True)
        else:
            line.update(report(args, rom, tim, K, ncell, value, nerr, mean_nexec, u_last, build_id,
                               soc0_all, tc_all, world))
            line["checks"]["hip_runtime"] = runtimes
            print(json.dumps(line), flush=True)


def report(args, rom, tim, K, ncell, value, nerr, mean_nexec, u_last, build_id, soc0_all, tc_all, world):
    """Rank 0's roofline / per-kernel / CPU-baseline objects (rank 0's shard timings)."""
    ncon = 4 * args.nc + 3 * args.np
    # boundzk is evaluated inside k_cell unless a k_bounds launch was timed
    bpc = algorithmic_bytes_per_cell(rom.NM, ncon, bool(args.bounds), Np=args.np, Nc=args.nc,
                                     bounds_kernel=tim.get("bounds", (0.0, 0))[1] > 0,
                                     plant_kernel=tim.get("plant", (0.0, 0))[1] > 0,
                                     hild_kernel=tim.get("hild", (0.0, 0))[1] > 0)
    # HIP-event averages over the sampled launches (--timing-every), so a kernel's share of
    # a step is its average x its launches per step.  k_flush flushes every cell each period
    # steps (the library default; every flush step is sampled); the rolling schedule
    # (MPCEKF_FLUSH_ROLL=1) flushes one slice of ncell / period cells every step on a second
    # stream beside k_bounds / Hildreth
    roll = os.environ.get("MPCEKF_FLUSH_ROLL", "0") != "0"
    # every flush step is sampled (--timing-every divides the flush period), so the sampled
    # flush launches are the timed region's flushes
    n_flush = K if roll else tim.get("flush", (0.0, 0))[1]
    period = int(os.environ.get("MPCEKF_FLUSH_PERIOD", str(LAZY_H)))  # the rolling schedule's slices
    cells_per_launch = {k: (ncell / period if (k == "flush" and roll) else ncell) for k in tim}
    per_kernel = {k: dict(ms_per_launch=tim[k][0] / max(tim[k][1], 1), launches_timed=tim[k][1],
                          launches=(n_flush if k == "flush" else K))
                  for k in tim if tim[k][1] > 0}
    for v in per_kernel.values():
        v["ms_total"] = v["ms_per_launch"] * v["launches"]
    # the dominant kernel = the largest share of the timed region (k_flush runs every 32 steps)
    dom = max(per_kernel, key=lambda k: per_kernel[k]["ms_total"])
    ms = per_kernel[dom]["ms_per_launch"]
    achieved = bpc[dom] * cells_per_launch[dom] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    pmc = {}
    if os.path.exists(args.pmc):
        try:
            with open(args.pmc) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            pmc = {}
    pmc_ok = pmc.get("build_id") == build_id and pmc.get("cells") == ncell and \
        pmc.get("Np", 5) == args.np and pmc.get("bounds", 1) == args.bounds and \
        pmc.get("rom_lookup", "linear") == args.rom_lookup
    traffic = pmc.get("per_launch_bytes", {}).get(dom) if pmc_ok else None
    flops = pmc.get("fp64_flops_per_launch", {}).get(dom) if pmc_ok else None
    fp64 = None
    if flops and ms > 0:
        tf = flops / (ms * 1e-3) / 1e12
        fp64 = {"achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                "flops_per_launch": flops, "source": os.path.relpath(args.pmc, ROOT)}
    cpu = None
    if world == 1 and not args.no_cpu:
        cpu = cpu_baseline(rom, soc0_all, tc_all, min(args.cpu_cells, ncell), args.cpu_steps or (args.warmup + K),
                           args.cpu_threads or cpu_threads_default(), Np=args.np, Nc=args.nc)
    return {
        "roofline": {
            "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": (os.path.relpath(args.pmc, ROOT) if traffic is not None else
                               f"null: {os.path.relpath(args.pmc, ROOT)} was not measured on this build "
                               f"({build_id}) and workload"),
            "algorithmic_bytes_per_cell": bpc[dom], "cells_per_launch": cells_per_launch[dom],
            "fp64": fp64,
            "step_equivalent": {
                "bytes_per_cell_step": survey_bytes_per_cell_step(rom.NM, ncon),
                "achieved": value * survey_bytes_per_cell_step(rom.NM, ncon) / 1e9, "unit": "GB/s",
                "note": "notional: SURVEY.md 8(d) eager-algorithm bytes x cell-steps/s; the deferred time "
                        "update does not move these bytes every step, so this is not achieved bandwidth",
            },
        },
        "kernels": {k: dict(ms_per_launch=round(v["ms_per_launch"], 5), launches=v["launches"],
                            launches_timed=v["launches_timed"],
                            ms_per_step=round(v["ms_total"] / K, 5) if K else None,
                            cells_per_launch=cells_per_launch[k],
                            gbs_algorithmic=round(bpc[k] * cells_per_launch[k] / (v["ms_per_launch"] * 1e-3) / 1e9, 1)
                            if v["ms_per_launch"] > 0 else None)
                    for k, v in per_kernel.items()},
        "cpu_baseline": cpu,
        "checks": {"cells_in_error": nerr, "mean_nexec": round(mean_nexec, 3), "build_id": build_id,
                   "u_last_mean_rank0": float(np.nanmean(u_last)) if u_last.size else None},
    }


if __name__ == "__main__":
    main()
