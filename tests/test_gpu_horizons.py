"""GPU parity over the full horizons of BASELINE.json's configs, bitwise against the
C oracle (oracle/mpcekf_oracle.c evaluates the kernels' defined arithmetic, asinh
included, so any difference is a bug).

  configs[1]  1 024 cells x 1 000 steps (+ warm-up 10), every cell
  configs[2]  65 536 cells x 1 000 steps, a 1/64 strided sample of cells checked
              (cells are independent, runMPC.m:83-112, so the oracle runs the sample alone)
  configs[4]  65 536 cells x 1 000 steps at Np = 20 / Nc = 10, a 1/32 sample (2 048 cells)
  and configs[1] / configs[2] / configs[4] again on the v3 (quintic) ROM the bench runs

The 1 000-step window covers the part of the charge where ~2 % of cells run
hildreth.m into maxIter (steps ~350-800).  The GPU runs in chunks of
250 steps (the deferred time update is call-boundary invariant, test_gpu_parity.py)
so only the sampled columns stay on the host.
"""
import os

import numpy as np
import pytest

from conftest import batch_inputs

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)  # the GPU box's CPU share


@pytest.fixture(scope="module")
def M(P):
    from importlib import import_module
    return import_module("mpc-ekf4fastcharge_amd.mpcekf")


def _bitwise(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
    if not same.all():
        i = tuple(np.argwhere(~same)[0])
        raise AssertionError(f"{what}: {int((~same).sum())} entries differ, first at (step, cell) {i}: "
                             f"{a[i]!r} vs {b[i]!r}")


def _gpu_sampled(M, rom, soc0, tc, steps, stride, cfg=None, chunk=250):
    keys = ("u", "v", "soc", "phise", "nexec")
    parts = {k: [] for k in keys}
    with M.Context(rom, len(soc0), cfg) as ctx:
        ctx.init_cells(soc0, tc)
        done = 0
        while done < steps:
            k = min(chunk, steps - done)
            o = ctx.step(k)
            for nm in keys:
                parts[nm].append(o[nm][:, ::stride].copy())
            del o
            done += k
        status = ctx.get_state()["status"][::stride]
    out = {k: np.concatenate(v) for k, v in parts.items()}
    out["status"] = status
    return out


def _check(out, ref):
    np.testing.assert_array_equal(out["status"], ref["status"])
    for k in ("u", "v", "soc", "phise", "nexec"):
        _bitwise(out[k], ref[k], k)


def test_configs1_1024_cells_1010_steps(rom, oc, M):
    soc0, tc = batch_inputs(1024)
    steps = 1010
    out = _gpu_sampled(M, rom, soc0, tc, steps, 1)
    ref = oc.run(rom, soc0, tc, steps, nthreads=NTHREADS)
    _check(out, ref)
    assert (out["nexec"] == 100).any()  # the maxIter window is inside the horizon


def test_configs2_65536_cells_1010_steps_sampled(rom, oc, M):
    soc0, tc = batch_inputs(65536)
    steps, stride = 1010, 64
    out = _gpu_sampled(M, rom, soc0, tc, steps, stride)
    ref = oc.run(rom, soc0[::stride], tc[::stride], steps, nthreads=NTHREADS)
    _check(out, ref)


@pytest.fixture(scope="module")
def rom_v3(P):
    return P.make_synth_rom(lookup="quintic")


@pytest.mark.parametrize("Np,Nc,stride", [(5, 2, 64), (20, 10, 16)])
def test_bench_workloads_on_the_v3_rom_sampled(rom_v3, oc, M, Np, Nc, stride):
    """The bench's own workloads — configs[2] (Np = 5) and configs[4] (Np = 20) on the v3
    quintic ROM bench.py runs by default — over the full 1,010-step window, sampled, bitwise
    against the C oracle."""
    soc0, tc = batch_inputs(65536)
    steps = 1010
    cfg = M.make_config(Np=Np, Nc=Nc)
    out = _gpu_sampled(M, rom_v3, soc0, tc, steps, stride, cfg=cfg)
    ref = oc.run(rom_v3, soc0[::stride], tc[::stride], steps, nthreads=NTHREADS, Np=Np, Nc=Nc)
    _check(out, ref)


def test_configs2_every_cell_on_the_v3_rom(rom_v3, oc, M):
    """configs[2] as bench.py runs it (65,536 cells, Np = 5, the v3 quintic ROM) over the full
    1,010-step window, every cell, bitwise against the C oracle (the sampled tests above hold
    1 in 64; this holds all of them: ~30 s of C oracle on the box's 16 host threads)."""
    soc0, tc = batch_inputs(65536)
    steps = 1010
    out = _gpu_sampled(M, rom_v3, soc0, tc, steps, 1)
    ref = oc.run(rom_v3, soc0, tc, steps, nthreads=NTHREADS)
    _check(out, ref)


def test_configs4_wide_65536_cells_1010_steps_sampled(rom, oc, M):
    soc0, tc = batch_inputs(65536)
    steps, stride = 1010, 32
    cfg = M.make_config(Np=20, Nc=10)
    out = _gpu_sampled(M, rom, soc0, tc, steps, stride, cfg=cfg)
    ref = oc.run(rom, soc0[::stride], tc[::stride], steps, nthreads=NTHREADS, Np=20, Nc=10)
    _check(out, ref)


def test_configs3_rank7_shard_131072_cells_sampled(rom, oc, M):
    """configs[3] (1,048,576 cells on 8 GPUs): the last rank's 131,072-cell shard of the
    global input sequence, as bench.py --gpus 8 --total-cells 1048576 assigns it, through
    one context on this GPU over the full 1,010-step window; a 1/64 sample (2,048 cells) bitwise."""
    import bench
    total, world, rank = 1048576, 8, 7
    soc0, tc = batch_inputs(total)
    a, b = bench.shard_range(total, world, rank)
    assert b - a == 131072
    steps, stride = 1010, 64
    out = _gpu_sampled(M, rom, soc0[a:b], tc[a:b], steps, stride)
    ref = oc.run(rom, soc0[a:b:stride], tc[a:b:stride], steps, nthreads=NTHREADS)
    _check(out, ref)


def test_configs1_every_cell_on_the_v3_rom(rom_v3, oc, M):
    """configs[1] as bench.py --cells-per-gpu 1024 runs it: 1,024 cells on the small-batch
    mappings (k_ekf4's lane quads, k_cell<P_MPC>, k_bounds beside k_hild on the side stream)
    with the v3 quintic ROM, every cell over the 1,010-step window, bitwise against the C
    oracle (test_configs1_1024_cells_1010_steps runs the v2 linear tables)."""
    soc0, tc = batch_inputs(1024)
    steps = 1010
    out = _gpu_sampled(M, rom_v3, soc0, tc, steps, 1)
    ref = oc.run(rom_v3, soc0, tc, steps, nthreads=NTHREADS)
    _check(out, ref)
    assert (out["nexec"] == 100).any()
