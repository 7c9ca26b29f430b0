"""GPU: small batches spread one wave per CU (round 5, mpcekf_kernels.hip spread_block).

Below 64 x #CUs x 4 cells the block-per-CU kernels (k_cell, k_hild, k_bounds) launch the
fewest 64-lane waves per block that still cover the batch in one round of blocks, instead
of 256-lane blocks packed four waves to a CU.  Each lane's arithmetic is its own, so the
results must be the packed launch's bits (MPCEKF_SPREAD=0) and the C oracle's, with ragged
last blocks (n not a multiple of 64) and the 4-lane-per-cell k_bounds at 64-thread blocks.
"""
import os

import numpy as np
import pytest

from conftest import batch_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(P):
    from importlib import import_module
    return import_module("mpc-ekf4fastcharge_amd.mpcekf")


def _run(M, rom, soc0, tc, steps, spread):
    old = os.environ.get("MPCEKF_SPREAD")
    os.environ["MPCEKF_SPREAD"] = "1" if spread else "0"
    try:
        with M.Context(rom, soc0.shape[0], M.make_config(bounds=True)) as ctx:
            ctx.init_cells(soc0, tc)
            return ctx.step(steps, outputs=("u", "v", "soc", "phise", "nexec", "zbk"))
    finally:
        if old is None:
            del os.environ["MPCEKF_SPREAD"]
        else:
            os.environ["MPCEKF_SPREAD"] = old


@pytest.mark.parametrize("n,lookup", [(1000, "quintic"), (77, "linear"), (5000, "quintic")])
def test_spread_equals_packed_and_oracle(P, M, oc, n, lookup):
    rom = P.make_synth_rom(lookup=lookup)
    soc0, tc = batch_inputs(n, seed=101 + n)
    steps = 40
    a = _run(M, rom, soc0, tc, steps, True)
    b = _run(M, rom, soc0, tc, steps, False)
    for k in ("u", "v", "soc", "phise", "nexec", "zbk"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    ref = oc.run(rom, soc0, tc, steps, nthreads=min(16, os.cpu_count() or 1))
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(a[k], ref[k], err_msg=k)


def test_quad_plant_with_temperature_profile(P, M, oc):
    """The lane-quad k_ekf4 with OB_step's simStep inside (quad_plant) under a per-step,
    per-cell temperature profile (the plant stores each step's TC for the EKF): the lane per
    cell k_cell path's bits and the C oracle's."""
    rom = P.make_synth_rom(lookup="quintic")
    n, steps = 300, 40
    soc0, tc = batch_inputs(n, seed=211)
    prof = tc[None, :] + 8.0 * np.sin(np.arange(steps)[:, None] / 7.0 + np.arange(n)[None, :] / 50.0)
    out = {}
    for quad in ("0", "1"):
        old = os.environ.get("MPCEKF_QUAD")
        os.environ["MPCEKF_QUAD"] = quad
        try:
            with M.Context(rom, n) as ctx:
                ctx.init_cells(soc0, tc)
                out[quad] = ctx.step(steps, tc=prof)
                out[quad]["state"] = ctx.get_state()
        finally:
            if old is None:
                del os.environ["MPCEKF_QUAD"]
            else:
                os.environ["MPCEKF_QUAD"] = old
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(out["0"][k], out["1"][k], err_msg=k)
    for k in ("ekf", "bigX", "scal", "lam"):
        np.testing.assert_array_equal(out["0"]["state"][k], out["1"]["state"][k], err_msg=k)
    ref = oc.run(rom, soc0, tc, steps, nthreads=min(16, os.cpu_count() or 1), tc_traj=prof)
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(out["1"][k], ref[k], err_msg=k)
