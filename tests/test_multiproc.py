"""CPU, world_size 2 over gloo: the multi-GPU decomposition of bench.py (contiguous
cell shards, no data-path collective, max-over-ranks timing) reproduces the
single-process result bit-for-bit (shard invariance)."""
import os
import sys

import numpy as np
import pytest

# torch is imported inside the tests and workers only: a GPU session collects this module
# too, and torch's bundled HIP runtime must never be mapped next to the library's
# (tests/test_gpu_runtime.py).

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, cpg, steps, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import importlib
    import bench
    import oracle_c
    P = importlib.import_module("mpc-ekf4fastcharge_amd")
    rom = P.make_synth_rom()
    soc0, tc = bench.batch_inputs(cpg * world - 5)       # ragged: shards of 22 and 21 cells
    lo, hi = bench.shard_range(cpg * world - 5, world, rank)
    out = oracle_c.run(rom, soc0[lo:hi], tc[lo:hi], steps, nthreads=1)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)       # bench.py's max-over-ranks timing
    u = torch.zeros((steps, cpg), dtype=torch.float64)
    u[:, :hi - lo] = torch.from_numpy(np.ascontiguousarray(out["u"]))
    gathered = [torch.empty_like(u) for _ in range(world)]
    dist.all_gather(gathered, u)
    if rank == 0:
        parts = [g[:, :b - a] for g, (a, b) in zip(gathered, [bench.shard_range(cpg * world - 5, world, r)
                                                                for r in range(world)])]
        q.put((float(t.item()), torch.cat(parts, dim=1).numpy()))
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_process(oc, rom):
    import bench
    import torch.multiprocessing as mp
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
    soc0, tc = bench.batch_inputs(cpg * world - 5)
    single = oc.run(rom, soc0, tc, steps, nthreads=2)
    np.testing.assert_array_equal(u_sharded, single["u"])


def test_bench_algorithmic_bytes():
    sys.path.insert(0, ROOT)
    import bench
    b = bench.algorithmic_bytes_per_cell(63, 23, True)
    # 416*NM state bytes, + model timestamps and the two input rings
    assert b["flush"] == 416 * 63 + 2 * 2 * 4 * 63 + 2 * 8 * bench.LAZY_H
    assert bench.survey_bytes_per_cell_step(63, 23) == 26736
    # the plant runs inside k_cell (no "plant" kernel) and boundzk comes from k_bounds' record
    assert "plant" not in b and set(b) == {"flush", "cell", "hild"}
    bk = bench.algorithmic_bytes_per_cell(63, 23, True, bounds_kernel=True)
    assert bk["bounds"] == (14 + 15 + 4 + 28) * 8
    # Np = 20 / Nc = 10: k_hild_prep hands k_hild_wide chol(E) (55) and K (100), not X (800 per cell)
    w = bench.algorithmic_bytes_per_cell(63, 100, True, Np=20, Nc=10)
    prob = 10 * 10 + 10 + 4 * 20 + 100 + 2
    assert w["hild"] == 2 * 8 * (36 + prob + 55 + 100) + 2 * 8 * 100 + 4 * 8


def test_shard_ranges_cover_the_batch():
    sys.path.insert(0, ROOT)
    import bench
    for total in (0, 1, 7, 1024, 1048576, 1048579):
        for world in (1, 2, 3, 8):
            r = [bench.shard_range(total, world, k) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            sizes = [b - a for a, b in r]
            assert max(sizes) - min(sizes) <= 1
    assert bench.shard_range(1048576, 8, 3) == (3 * 131072, 4 * 131072)   # configs[3]


def _bench(*args, env=None):
    import json
    import subprocess
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=e, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0], r.stderr


@pytest.mark.parametrize("gpus,extra,total,per", [
    (2, [], 131072, [65536, 65536]),
    (3, ["--cells-per-gpu", "1000"], 3000, [1000, 1000, 1000]),
    (8, ["--total-cells", "1048576"], 1048576, [131072] * 8),     # configs[3]
    (3, ["--total-cells", "1000"], 1000, [334, 333, 333]),
])
def test_bench_spawns_ranks_over_gloo(gpus, extra, total, per):
    """bench.py --gpus N without torchrun starts N rank processes (here with --dry-run:
    gloo collectives, no GPU); each prints its contiguous cell range, rank 0 prints the
    one JSON line with n_gpus = N and the whole-job cell count."""
    line, err = _bench("--gpus", str(gpus), "--dry-run", "--steps", "3", *extra)
    assert line["n_gpus"] == gpus and line["dry_run"] is True
    assert line["config"]["total_cells"] == total and line["config"]["cells_per_gpu"] == per
    assert line["scaling"] == ("strong" if "--total-cells" in extra else "weak")
    for r in range(gpus):
        assert f"rank {r}/{gpus}: cells [" in err


def test_bench_refuses_world_size_mismatch():
    import subprocess
    e = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, env=e, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_bench_force_dist_at_world_size_one():
    """--force-dist creates the gloo process group at WORLD_SIZE 1 (the timing coordinator
    on a one-GPU box; here with --dry-run) and runs the timing collectives through it; without it
    a single rank runs no collective."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    line, err = _bench("--gpus", "1", "--dry-run", "--force-dist", "--steps", "3", env=env)
    assert "process group: gloo" in err and line["config"]["timing_collectives"] == "gloo"
    line, err = _bench("--gpus", "1", "--dry-run", "--steps", "3")
    assert "process group: none" in err and line["config"]["timing_collectives"] == "none"
    # outside a launcher (no RANK / MASTER_*): the coordinator makes a world of one itself
    line, err = _bench("--gpus", "1", "--dry-run", "--force-dist", "--steps", "3")
    assert "process group: gloo" in err and line["config"]["timing_collectives"] == "gloo"
