"""BASELINE.json configs[3] on the one leased GPU: 1,048,576 cells, Np = 5 / Nc = 2.

On the 8-GPU node bench.py --gpus 8 --total-cells 1048576 gives each rank a contiguous
131,072-cell shard (bench.shard_range).  Here every one of the eight shards runs through
the library in turn, over the 1,010-step window that holds the maxIter regime, and the
whole 1,048,576-cell input also runs as ONE context (≈17 GB of state, well inside one
MI355X's 288 GB).  Checks:

  * each shard's 1/64 sample of cells (16,384 of the million over the eight) is bitwise equal to the C oracle;
  * the concatenation of the eight shards' samples equals the single-context run's
    sample, bit for bit (runMPC.m:83-112 has no cross-cell term, so the shard boundaries
    cannot change any cell's bits).

Outputs go to library-allocated device buffers in 101-step chunks; only the sampled
columns come back (pitched copies).
"""
import os

import numpy as np
import pytest

from conftest import batch_inputs

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)
TOTAL, WORLD, STEPS, STRIDE, CHUNK = 1048576, 8, 1010, 64, 101
KEYS = ("u", "v", "soc", "phise", "nexec")


@pytest.fixture(scope="module")
def M(P):
    from importlib import import_module
    return import_module("mpc-ekf4fastcharge_amd.mpcekf")


def _run_sampled(M, rom, soc0, tc):
    """One context over these cells, STEPS steps, device outputs (library-allocated
    buffers); the STRIDE-sampled columns of every store plus the final status, on the
    host."""
    n = len(soc0)
    bufs = [M.DeviceBuffer((CHUNK, n), np.float64) for _ in range(4)] + [M.DeviceBuffer((CHUNK, n), np.int32)]
    parts = {k: [] for k in KEYS}
    try:
        with M.Context(rom, n, None) as ctx:
            ctx.init_cells(soc0, tc)
            done = 0
            while done < STEPS:
                k = min(CHUNK, STEPS - done)
                ctx.step_device(k, *bufs)
                ctx.sync()
                for nm, b in zip(KEYS, bufs):
                    parts[nm].append(b.sampled(k, STRIDE))
                done += k
            status = ctx.get_state()["status"][::STRIDE]
    finally:
        for b in bufs:
            b.free()
    out = {k: np.concatenate(v) for k, v in parts.items()}
    out["status"] = status
    return out


def _bitwise(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
    if not same.all():
        i = tuple(np.argwhere(~same)[0])
        raise AssertionError(f"{what}: {int((~same).sum())} entries differ, first at {i}: {a[i]!r} vs {b[i]!r}")


def test_configs3_all_eight_shards_and_single_context(rom, oc, M):
    import bench
    soc0, tc = batch_inputs(TOTAL)
    shard_out = []
    for rank in range(WORLD):
        a, b = bench.shard_range(TOTAL, WORLD, rank)
        assert b - a == TOTAL // WORLD and a % STRIDE == 0
        out = _run_sampled(M, rom, soc0[a:b], tc[a:b])
        ref = oc.run(rom, soc0[a:b:STRIDE], tc[a:b:STRIDE], STEPS, nthreads=NTHREADS)
        np.testing.assert_array_equal(out["status"], ref["status"])
        for k in KEYS:
            _bitwise(out[k], ref[k], f"shard {rank}: {k}")
        shard_out.append(out)
    assert any((o["nexec"] == 100).any() for o in shard_out)  # the maxIter window is inside
    whole = _run_sampled(M, rom, soc0, tc)
    for k in KEYS + ("status",):
        cat = np.concatenate([o[k] for o in shard_out], axis=-1)
        _bitwise(whole[k], cat, f"single context vs concatenated shards: {k}")
