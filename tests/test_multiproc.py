"""CPU, world_size 2 over gloo: the multi-GPU decomposition of bench.py (contiguous
cell shards, no data-path collective, max-over-ranks timing) reproduces the
single-process result bit-for-bit (shard invariance)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, cpg, steps, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import importlib
    import bench
    import oracle_c
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    rom = P.make_synth_rom()
    soc0, tc = bench.batch_inputs(cpg * world)
    sl = slice(rank * cpg, (rank + 1) * cpg)
    out = oracle_c.run(rom, soc0[sl], tc[sl], steps, nthreads=1)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)       # bench.py's max-over-ranks timing
    u = torch.from_numpy(np.ascontiguousarray(out["u"]))
    gathered = [torch.empty_like(u) for _ in range(world)]
    dist.all_gather(gathered, u)
    if rank == 0:
        q.put((float(t.item()), torch.cat(gathered, dim=1).numpy()))
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_process(oc, rom):
    import bench
    world, cpg, steps = 2, 24, 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, cpg, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, u_sharded = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    soc0, tc = bench.batch_inputs(cpg * world)
    single = oc.run(rom, soc0, tc, steps, nthreads=2)
    np.testing.assert_array_equal(u_sharded, single["u"])


def test_bench_algorithmic_bytes():
    sys.path.insert(0, ROOT)
    import bench
    b = bench.algorithmic_bytes_per_cell(63, 23, True)
    # 416*NM state bytes, + model timestamps and the two input rings
    assert b["flush"] == 416 * 63 + 2 * 2 * 4 * 63 + 2 * 8 * 32
    assert bench.survey_bytes_per_cell_step(63, 23) == 26736
