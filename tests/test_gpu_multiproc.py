"""Multi-process runs through the library on the one leased GPU: the multi-GPU
decomposition (one process + one context per device, contiguous cell shards, no
data-path collective; runMPC.m:83-112 has no cross-cell term) with both ranks on
device 0.  The 8-GPU case itself is the driver's; this checks its mechanics."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _clean_env():
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


def test_two_processes_two_contexts_bit_identical(tmp_path, rom, P):
    from importlib import import_module
    sys.path.insert(0, ROOT)
    import bench
    M = import_module("mpc-ekf4fastcharge_amd.mpcekf")
    total, steps, world = 3001, 120, 2           # ragged shards: 1501 + 1500 cells
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "shard_worker.py"), "--rank", str(r),
                               "--world", str(world), "--total", str(total), "--steps", str(steps),
                               "--out", str(tmp_path / f"r{r}.npz")], env=_clean_env())
             for r in range(world)]
    codes = [p.wait(timeout=240) for p in procs]
    assert codes == [0, 0]
    parts = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert [(int(p["lo"]), int(p["hi"])) for p in parts] == [bench.shard_range(total, world, r) for r in range(world)]
    soc0, tc = bench.batch_inputs(total)
    single = M.runMPC(rom, soc0, tc, steps)
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(np.concatenate([p[k] for p in parts], axis=1), single[k], err_msg=k)
    np.testing.assert_array_equal(np.concatenate([p["status"] for p in parts]), single["status"])


def test_bench_two_ranks_share_device():
    """bench.py --gpus 2 (its own rank launcher) with both ranks on device 0 and gloo
    timing collectives: n_gpus = 2, both shards run through the library, max-over-ranks
    time, per-rank cell ranges printed."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--cells-per-gpu", "4096", "--steps", "40", "--warmup", "4", "--no-cpu"],
                       capture_output=True, text=True, env=_clean_env(), timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["total_cells"] == 8192
    assert line["config"]["cells_per_gpu"] == [4096, 4096]
    assert line["checks"]["cells_in_error"] == 0 and line["value"] > 0
    assert "rank 0/2: cells [0, 4096)" in r.stderr and "rank 1/2: cells [4096, 8192)" in r.stderr
