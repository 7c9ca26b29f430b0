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
    # the library default: the plant inside k_cell (no "plant" kernel), boundzk in k_bounds
    # from k_cell's hand-off record
    assert "plant" not in b and set(b) == {"flush", "cell", "hild", "bounds"}
    assert b["bounds"] == (14 + 15 + 4 + 28) * 8
    # boundzk inside k_cell (MPCEKF_CELL_BOUNDS=1): no record, corner 1's Sigma + boundzk in k_cell
    bc = bench.algorithmic_bytes_per_cell(63, 23, True, bounds_kernel=False)
    assert set(bc) == {"flush", "cell", "hild"} and bc["cell"] == b["cell"] - 14 * 8 + 15 * 8 + 28 * 8
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


def test_bench_rank_path_reduces_over_gloo_and_parent_maps_no_runtime(tmp_path):
    """bench.py --gpus 2 (no torchrun): the parent counts nothing through HIP or torch and
    maps no GPU runtime before it spawns the ranks (MPCEKF_BENCH_PARENT_MAPS records its
    /proc/self/maps runtime lines), and the two ranks' gloo coordinators reduce the timing
    as max over ranks and the shard coverage as sums: every cell once, the full SOC0
    checksum (ragged shards of 1,001 cells)."""
    import bench
    maps = tmp_path / "parent_maps.txt"
    line, err = _bench("--gpus", "2", "--dry-run", "--total-cells", "1001", "--steps", "3",
                       env={"MPCEKF_BENCH_PARENT_MAPS": str(maps)})
    assert maps.exists() and maps.read_text().strip() == ""
    chk = line["dry_run_checks"]
    assert chk["cells"] == 1001 and line["config"]["cells_per_gpu"] == [501, 500]
    soc0, _ = bench.batch_inputs(1001)
    assert abs(chk["soc0_sum"] - soc0.sum()) <= 1e-9 * soc0.sum()
    assert chk["max_dt_s"] >= 0.04          # rank 1's 40 ms, not rank 0's 20 ms
    assert line["config"]["timing_collectives"] == "gloo"


def test_count_gpus_from_kfd_topology(tmp_path):
    """The launcher's device count (no HIP, no torch): KFD GPU nodes with an accessible
    render node, limited by the *_VISIBLE_DEVICES lists."""
    import bench
    sysfs, dev = tmp_path / "nodes", tmp_path / "dri"
    dev.mkdir()
    for i, (simd, minor) in enumerate([(0, 0), (256, 128), (256, 136), (256, 144), (256, 152)]):
        d = sysfs / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndrm_render_minor {minor}\n")
    for minor in (128, 136, 144):           # renderD152 is not in this container
        (dev / f"renderD{minor}").write_text("")
    assert bench.count_gpus(str(sysfs), str(dev), env={}) == 3
    assert bench.count_gpus(str(sysfs), str(dev), env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.count_gpus(str(sysfs), str(dev), env={"ROCR_VISIBLE_DEVICES": "2"}) == 1
    assert bench.count_gpus(str(tmp_path / "none"), str(dev), env={}) == 0


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
