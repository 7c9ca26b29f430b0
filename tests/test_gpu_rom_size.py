"""GPU parity at the SURVEY §6 ROM-size sensitivity points (NM = 21 and NM = 147).

Up to NM ~ 75 (default 101 x 6 electrode grid) the model rows of both ROM blobs sit in
LDS next to the electrode tables.  Above that the host switches the kernels to the
rom_global layout (KRom::rom_global): only the tables are staged, the model rows are read
from the global blob.  The arithmetic is the same, so every comparison with the C oracle
is bitwise, as in test_gpu_parity.py.  MPCEKF_ROM_GLOBAL=1 forces the global layout at
any NM, which pins it against the LDS layout on the same inputs.
"""
import numpy as np
import pytest

from conftest import batch_inputs
from test_gpu_parity import _bitwise, _run_with_env

pytestmark = pytest.mark.gpu

TRAJ = ("u", "v", "soc", "phise", "nexec", "x", "zk", "zbk", "J_unc", "J_fin", "norm_du", "nviol")
REF = dict(u="u", v="v", soc="soc", phise="phise", nexec="nexec", x="x", zk="zk_traj", zbk="zbk_traj",
           J_unc="J_unc", J_fin="J_fin", norm_du="norm_du", nviol="nviol")


@pytest.fixture(scope="module")
def M(P):
    from importlib import import_module
    return import_module("mpc-ekf4fastcharge_amd.mpcekf")


def _rom(P, temps, socs):
    return P.make_synth_rom(T_degC=tuple(np.linspace(15.0, 35.0, temps)),
                            SOC_pct=tuple(np.linspace(0.0, 100.0, socs)))


@pytest.mark.parametrize("temps,socs,method", [(7, 21, "OB"), (7, 21, "MB"), (1, 21, "OB")])
def test_rom_size_sensitivity_matches_oracle(P, oc, M, temps, socs, method):
    """NM = 147 (rom_global layout) and NM = 21 (LDS layout): closed loop with boundzk and
    every runMPC.m store, bitwise against the C oracle."""
    rom = _rom(P, temps, socs)
    assert rom.NM == temps * socs
    n, steps = 96, 200
    soc0, tc = batch_inputs(n, seed=41)
    soc0[3] = 130.0                      # an error / lock-out cell
    cfg = M.make_config(method=method, bounds=True)
    with M.Context(rom, n, cfg) as ctx:
        ctx.init_cells(soc0, tc)
        out = ctx.step(steps, outputs=TRAJ)
        st = ctx.get_state()
    ref = oc.run(rom, soc0, tc, steps, nthreads=8, traj=True, method=method)
    for k, rk in REF.items():
        _bitwise(out[k], ref[rk], f"NM={rom.NM} {method} {k}")
    np.testing.assert_array_equal(st["status"], ref["status"])


def test_rom_global_layout_matches_lds_layout(P, oc, M):
    """MPCEKF_ROM_GLOBAL=1 at NM = 63 gives the LDS layout's bits, state included, through
    k_cell, the lane-quad k_ekf4 (MPCEKF_QUAD=1) and k_bounds; every run is the C
    oracle's trajectory."""
    rom = P.make_synth_rom()
    n = 640
    soc0, tc = batch_inputs(n, seed=43)
    ref = oc.run(rom, soc0, tc, 150, nthreads=8)
    for quad in (0, 1):
        a = _run_with_env(M, rom, soc0, tc, 150, MPCEKF_QUAD=quad, MPCEKF_ROM_GLOBAL=0)
        b = _run_with_env(M, rom, soc0, tc, 150, MPCEKF_QUAD=quad, MPCEKF_ROM_GLOBAL=1)
        for k in ("u", "v", "soc", "phise", "nexec"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"quad={quad} {k}")
            _bitwise(b[k], ref[k], f"quad={quad} {k}")
        for k in ("ekf", "bigX", "scal", "lam"):
            np.testing.assert_array_equal(a["state"][k], b["state"][k], err_msg=f"quad={quad} {k}")


def test_rom_global_stage_entry_points(P, M):
    """The stage entry points (OB_step / iterEKF with boundzk / EKFmatsHandler / iterMPC)
    at NM = 147 give the fused step's bits."""
    rom = _rom(P, 7, 21)
    n, steps = 64, 15
    soc0, tc = batch_inputs(n, seed=47)
    fused = M.runMPC(rom, soc0, tc, steps)
    with M.Context(rom, n) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)
        for k in range(steps):
            v = ctx.OB_step(uk)
            zk, zb, xind = ctx.iterEKF(v, uk)
            assert np.isfinite(zb).any()
            lin = ctx.EKFmatsHandler(zk, xind)
            uk, ne = ctx.iterMPC(lin, zk[:, -1])
            np.testing.assert_array_equal(v, fused["v"][k])
            np.testing.assert_array_equal(uk, fused["u"][k])
            np.testing.assert_array_equal(ne, fused["nexec"][k])


def test_largest_grid_matches_oracle_and_beyond_is_refused(P, oc, M):
    """The largest set-point grid the kernels take (MAXT x MAXZ = 8 x 40, NM = 320) runs
    bitwise against the C oracle; one temperature more is MPCEKF_E_UNSUPPORTED with a
    message, never a silent fallback."""
    rom = _rom(P, 8, 40)
    n, steps = 32, 40
    soc0, tc = batch_inputs(n, seed=53)
    out = M.runMPC(rom, soc0, tc, steps)
    ref = oc.run(rom, soc0, tc, steps, nthreads=8)
    for k in ("u", "v", "soc", "phise", "nexec"):
        _bitwise(out[k], ref[k], f"NM=320 {k}")
    with pytest.raises(Exception, match="exceeds"):
        M.Context(_rom(P, 9, 21), 8)
