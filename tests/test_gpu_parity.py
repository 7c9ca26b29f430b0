"""GPU parity: the HIP path (through the C-ABI) against the C oracle.

Tolerances.  The kernels evaluate the same defined operation order as
oracle/mpcekf_oracle.c (explicit fma, ascending sums from +0.0, asinh spelled
out as dasinh/orc_asinh on both sides), so every comparison with the C oracle
is BITWISE (NaN patterns included).  Against the numpy restatement's golden
fixtures (LAPACK, libm asinh) the north_star bar 1e-6 relative applies, or
1e-9 where the fixture stays well conditioned.
"""
import numpy as np
import pytest

from conftest import batch_inputs

pytestmark = pytest.mark.gpu

RTOL_TIGHT = 1e-9
RTOL_NORTH_STAR = 1e-6


def _rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    both_nan = np.isnan(a) & np.isnan(b)
    d = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    d[both_nan] = 0.0
    d[np.isnan(d)] = np.inf
    return d


@pytest.fixture(scope="module")
def M(P):
    from importlib import import_module
    m = import_module("mpc-ekf4fastcharge_amd.mpcekf")
    return m


def test_closed_loop_matches_oracle(rom, oc, M):
    n, steps = 96, 400
    soc0, tc = batch_inputs(n)
    soc0[0], tc[0] = 10.0, 25.0          # the golden runMPC.m cell
    ref = oc.run(rom, soc0, tc, steps, nthreads=8)
    out = M.runMPC(rom, soc0, tc, steps)
    for k in ("u", "v", "soc", "phise", "nexec"):
        _bitwise(out[k], ref[k], k)


def _bitwise(a, b, what=""):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
    if not same.all():
        i = np.argwhere(~same)[0]
        raise AssertionError(f"{what}: {int((~same).sum())} entries differ, first at {tuple(i)}: "
                             f"{a[tuple(i)]!r} vs {b[tuple(i)]!r} (max rel {_rel(a, b).max():.3e})")


def _agree_steps(ref, g, rtol):
    """Number of leading steps on which two trajectory sets agree to rtol (u, v, soc, phise)."""
    bad = np.zeros(g["u"].shape[0], dtype=bool)
    for k in ("u", "v", "soc", "phise"):
        r = _rel(ref[k], g[k])
        bad |= (r > rtol).reshape(r.shape[0], -1).any(axis=1)
    return int(np.argmax(bad)) if bad.any() else int(bad.shape[0])


@pytest.mark.parametrize("lookup,quad", [("linear", "1"), ("quintic", "1"), ("quintic", "0")])
def test_lockout_and_error_cells(P, oc, M, lookup, quad):
    # SOC0 = 130 % drives getVariables' clamps every call -> warnCount > 10 -> lock-out; on the
    # v3 ROM the locked-out cells' NaN states reach the branch-free lookups; quad: the small-batch
    # lane-quad path (the default at 4 cells) or the lane per cell k_cell
    rom = P.make_synth_rom(lookup=lookup)
    soc0 = np.array([10.0, 130.0, 20.0, 130.0])
    tc = np.array([25.0, 25.0, 15.0, 35.0])
    steps = 30
    ref = oc.run(rom, soc0, tc, steps, nthreads=1)
    out = _run_with_env(M, rom, soc0, tc, steps, MPCEKF_QUAD=quad)
    status = out["state"]["status"]
    assert np.array_equal(status, ref["status"])
    assert (status[[1, 3]] & 1).all()
    for k in ("u", "v", "soc", "phise"):
        _bitwise(out[k], ref[k], k)


def test_stage_entry_points_match_fused(rom, M):
    """OB_step -> iterEKF -> EKFmatsHandler -> iterMPC through the stage ABI equals
    the fused step (same kernels, same state)."""
    n, steps = 256, 25
    soc0, tc = batch_inputs(n, seed=7)
    fused = M.runMPC(rom, soc0, tc, steps)
    with M.Context(rom, n) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)
        for k in range(steps):
            v = ctx.OB_step(uk)
            zk, zb, xind = ctx.iterEKF(v, uk)
            lin = ctx.EKFmatsHandler(zk, xind)
            ph = (lin[:, 20:26] * lin[:, 29:35]).sum(1)  # informative only
            uk, ne = ctx.iterMPC(lin, zk[:, -1])
            np.testing.assert_array_equal(v, fused["v"][k])
            np.testing.assert_array_equal(uk, fused["u"][k])
            np.testing.assert_array_equal(zk[:, -1], fused["soc"][k])
            np.testing.assert_array_equal(ne, fused["nexec"][k])
            del ph


def test_predmat_hildreth_match_oracle(rom, oc, M):
    rng = np.random.default_rng(3)
    n = 300
    a = np.concatenate([rng.uniform(0.3, 0.999, (n, 5)), np.ones((n, 1))], 1)
    Cr = np.concatenate([rng.normal(0, 1e-3, (n, 5)), np.zeros((n, 1))], 1)
    D = rng.normal(0, 1e-3, n)
    Phi, G = M.predMat(a, Cr, D, 5, 2)
    for i in range(0, n, 37):
        P2, G2 = oc.predmat(a[i], Cr[i], D[i], 5, 2)
        np.testing.assert_array_equal(Phi[i], P2)
        np.testing.assert_array_equal(G[i], G2)
    # random strictly convex QPs with the 23-row constraint shape
    E = np.empty((n, 2, 2))
    F = rng.normal(0, 1, (n, 2))
    Mm = rng.normal(0, 1, (n, 23, 2))
    g = rng.normal(0.5, 1, (n, 23))
    for i in range(n):
        A = rng.normal(0, 1, (2, 2))
        E[i] = A @ A.T + 0.5 * np.eye(2)
        E[i] = (E[i] + E[i].T) / 2
    lam0 = np.abs(rng.normal(0, 0.1, (n, 23)))
    DU, lam, ne = M.hildreth(E, F, Mm, g, lam0, 100)
    for i in range(n):
        d2, l2, k2 = oc.hildreth(E[i], F[i], Mm[i], g[i], lam0[i], 100)
        assert ne[i] == k2
        np.testing.assert_array_equal(DU[i], d2)
        np.testing.assert_array_equal(lam[i], l2)


def test_full_size_properties(rom, M):
    """65 536 cells x 20 steps: finite outputs, SOC increases under charge, no error bits,
    constraints respected where Hildreth converged, result independent of batch split."""
    n, steps = 65536, 20
    soc0, tc = batch_inputs(n)
    out = M.runMPC(rom, soc0, tc, steps)
    assert (out["status"] == 0).all()
    for k in ("u", "v", "soc", "phise"):
        assert np.isfinite(out[k]).all(), k
    assert (np.diff(out["soc"], axis=0) >= -1e-12).all()
    assert (out["u"] >= -rom.Q * 2 - 1e-6).all()
    # shard invariance: a contiguous slice run alone gives identical bits
    sl = slice(12345, 12345 + 1000)
    part = M.runMPC(rom, soc0[sl], tc[sl], steps)
    for k in ("u", "v", "soc", "phise"):
        np.testing.assert_array_equal(part[k], out[k][:, sl])


def _golden(name):
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))


@pytest.mark.parametrize("fixture,romkw,rtol", [
    ("batch8_200", {}, 1e-9),
    ("rom_nt1_200", dict(T_degC=(25.0,)), 1e-9),
    ("edge_cells_400", {}, 1e-8),
])
def test_gpu_matches_golden_fixtures(P, M, fixture, romkw, rtol):
    """Against the MATLAB-faithful numpy restatement (tests/golden, tools/make_golden.py)."""
    g = _golden(fixture)
    rom = P.make_synth_rom(**romkw)
    out = M.runMPC(rom, g["soc0"], g["tc"], g["u"].shape[0])
    np.testing.assert_array_equal(out["status"], g["status"])
    for k in ("u", "v", "soc", "phise"):
        assert _rel(out[k], g[k]).max() <= rtol, k
    np.testing.assert_array_equal(out["nexec"], g["nexec"])


def test_zk_and_boundzk_match_oracle(rom, oc, M):
    n, steps = 40, 60
    soc0, tc = batch_inputs(n, seed=11)
    ref = oc.run(rom, soc0, tc, steps, nthreads=4, want_zk=True)
    cfg = M.make_config(bounds=True)
    with M.Context(rom, n, cfg) as ctx:
        ctx.init_cells(soc0, tc)
        ctx.step(steps)
        zk, zb = ctx.get_zk()
    _bitwise(zk, ref["zk"], "zk")
    _bitwise(zb, ref["zbk"], "boundzk")


def test_checkpoint_restore_is_exact(rom, oc, M):
    """get_state / set_state mid-run: the rerun from the checkpoint gives the first run's
    bits, and both are the C oracle's uninterrupted trajectory (steps 15-40)."""
    n = 2048
    soc0, tc = batch_inputs(n, seed=5)
    with M.Context(rom, n) as ctx:
        ctx.init_cells(soc0, tc)
        ctx.step(15)
        snap = ctx.get_state()
        a = ctx.step(25)
        ctx.set_state(snap)
        b = ctx.step(25)
    ref = oc.run(rom, soc0, tc, 40, nthreads=8)
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(a[k], b[k])
        _bitwise(b[k], ref[k][15:], k)


def test_runmpc_cell_full_charge(rom, oc, M):
    """configs[0]: the runMPC.m cell (SOC0 = 10 %, 25 degC), all 3001 steps.

    Bitwise against the C oracle over the whole charge.  Against the numpy golden
    (LAPACK / libm arithmetic) within north_star's 1e-6 up to the step where the two
    restatements themselves part: from ~2,900 on, hildreth.m runs into maxIter on
    infeasible QPs every step and ulp-level differences grow to O(1)
    (tests/test_oracle.py::test_tail_is_ill_conditioned shows a 1-ulp change of SOC0
    does the same), so no implementation can be held to 1e-6 there."""
    g = _golden("runmpc_soc10_tc25")
    out = M.runMPC(rom, g["soc0"], g["tc"], 3001)
    ref = oc.run(rom, g["soc0"], g["tc"], 3001, nthreads=1)
    for k in ("u", "v", "soc", "phise", "nexec"):
        _bitwise(out[k], ref[k], k)
    agree = _agree_steps(ref, g, RTOL_NORTH_STAR)
    assert agree >= 2900, agree
    for k in ("u", "v", "soc", "phise"):
        assert _rel(out[k][:agree], g[k][:agree]).max() <= RTOL_NORTH_STAR, k


def test_runmpc_tail_inside_ulp_envelope(rom, M):
    """configs[0]'s last ~200 steps, where the single numpy fixture cannot hold any
    implementation (test_runmpc_cell_full_charge): the GPU trajectory lies inside the
    per-step envelope of the MATLAB-faithful restatement's ulp ensemble (SOC0 -8..+8 ulps,
    and 32 members with a random -1..1 ulp kick of the command every step) widened by
    north_star's 1e-6, at every step of 2,800-3,001, and reaches 90 % SOC at the step the
    ensemble does (tests/envelope.py; tools/make_golden.py make_envelopes)."""
    import envelope
    out = M.runMPC(rom, np.array([10.0]), np.array([25.0]), 3001)
    envelope.check_run(out, envelope.load("env_runmpc_3001"))


def test_wide_near_limit_tails_in_ensemble_distribution(rom, M):
    """The Np = 20 near-limit cells over steps 25-200 (the dense-H fixture test holds only
    the first 25 of three cells): their closed loops are chaotic, so the GPU's window mean,
    10th / 90th percentiles of u, v, soc, phise and final SOC are held inside the range of
    the same statistics over the MATLAB-faithful restatement's 25-member ulp ensemble
    (tests/envelope.py)."""
    import envelope
    w = envelope.load("env_wide_near4_200")
    out = M.runMPC(rom, w["soc0"], w["tc"], 200, cfg=M.make_config(Np=20, Nc=10))
    envelope.check_near(out, w)


def test_deferred_time_update_is_schedule_invariant(rom, M):
    """The fused step defers the all-model time update (ring of LAZY_H = 64 inputs,
    flush every 64 steps and at the end of each call).  Splitting the same run into
    calls that straddle the flush boundaries must give bit-identical trajectories
    and an identical full state (every local model's record and plant state)."""
    n = 2048
    soc0, tc = batch_inputs(n, seed=9)
    chunks = [1, 31, 32, 33, 53, 63, 64, 65, 250]
    with M.Context(rom, n) as a, M.Context(rom, n) as b:
        a.init_cells(soc0, tc)
        b.init_cells(soc0, tc)
        ra = a.step(sum(chunks))
        rb = [b.step(k) for k in chunks]
        sa, sb = a.get_state(), b.get_state()
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(ra[k], np.concatenate([r[k] for r in rb]), err_msg=k)
    for k in ("bigX", "ekf", "scal", "lam", "warn", "status"):
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)


def _run_with_env(M, rom, soc0, tc, steps, **env):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        with M.Context(rom, len(soc0)) as ctx:   # the overrides are read at context creation
            ctx.init_cells(soc0, tc)
            out = ctx.step(steps)
            out["state"] = ctx.get_state()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out


def test_flush_period_is_exact(rom, M):
    """The deferred time update gives the same bits for any flush period <= the ring, with
    every cell flushed at once on the step's stream (the default) and with the rolling
    schedule (MPCEKF_FLUSH_ROLL=1: one cell slice per step on a second stream)."""
    n = 1000  # slices of unequal size for P = 7, 32 and 64
    soc0, tc = batch_inputs(n, seed=22)
    runs = [_run_with_env(M, rom, soc0, tc, 300, MPCEKF_FLUSH_PERIOD=p, MPCEKF_FLUSH_ROLL=roll)
            for p, roll in ((64, 0), (1, 0), (7, 0), (32, 0), (64, 1), (7, 1))]
    for r in runs[1:]:
        for k in ("u", "v", "soc", "phise", "nexec"):
            np.testing.assert_array_equal(r[k], runs[0][k], err_msg=k)
        for k in ("ekf", "bigX"):
            np.testing.assert_array_equal(r["state"][k], runs[0]["state"][k], err_msg=k)


def test_mpc_stage_edge_records(rom, oc, M):
    """iterMPC (Np = 5, k_cell's MPC part + k_hild / k_hild_slow) on linearisation records
    built to leave the fast rank-2 sweep, next to plain ones: overflowing and infinite G
    rows, H_ii outside [2^-400, 2^400], a NaN bound.  uk, nexec and lambda bitwise against
    the oracle (NaN where the oracle has NaN)."""
    n = 64
    soc0, tc = batch_inputs(n, seed=51)
    with M.Context(rom, n) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)
        for _ in range(4):
            v = ctx.OB_step(uk)
            zk, _, xind = ctx.iterEKF(v, uk)
            lin = ctx.EKFmatsHandler(zk, xind)
            uk, _ = ctx.iterMPC(lin, zk[:, -1])
        v = ctx.OB_step(uk)
        zk, _, xind = ctx.iterEKF(v, uk)
        lin = np.array(ctx.EKFmatsHandler(zk, xind), dtype=np.float64)
        g = np.arange(n) % 8
        lin[g == 1, 13:19] *= 1e300   # Cv: G_v rows overflow
        lin[g == 2, 19] = 1e200        # Dv: H_ii overflows
        lin[g == 3, 20:26] = np.inf    # Cphi: G_e rows non-finite
        lin[g == 4, 27] = np.nan       # bv: a NaN bound
        lin[g == 5, 13:20] *= 1e-170   # G_v rows tiny: H_ii below 2^-400
        zend = zk[:, -1]
        st = ctx.get_state()
        uk_r, ne_r, _, lam_r = oc.mpc_lin(rom, lin, zend, st["scal"][:, 5], st["lam"])
        uk, ne = ctx.iterMPC(lin, zend)
        lam = ctx.get_state()["lam"]
    for k, (a, b) in {"uk": (uk, uk_r), "lam": (lam, lam_r)}.items():
        assert np.array_equal(a, b, equal_nan=True), (k, np.nonzero(~((a == b) | (np.isnan(a) & np.isnan(b))))[0][:8])
    np.testing.assert_array_equal(ne, ne_r)


def test_bounds_side_stream_is_exact(rom, M):
    """k_bounds on a second stream beside Hildreth (MPCEKF_BOUNDS_SIDE, an option since
    round 6; up to 16,384 cells by default before) joins it before k_flush / the next k_cell rewrite the
    records it reads: boundzk and the loop give the bits of k_bounds on the step's stream,
    over two flush windows, with per-kernel timing on (its events straddle the streams)."""
    import os
    n = 1000
    soc0, tc = batch_inputs(n, seed=23)
    outs = []
    for side in ("0", "1000000"):
        old = os.environ.get("MPCEKF_BOUNDS_SIDE")
        os.environ["MPCEKF_BOUNDS_SIDE"] = side
        try:
            with M.Context(rom, n, M.make_config(bounds=True)) as ctx:
                ctx.init_cells(soc0, tc)
                ctx.set_timing(True)
                out = ctx.step(140, outputs=("u", "v", "zk", "zbk"))
                out["state"] = ctx.get_state()
                out["timing"] = ctx.get_timing()
        finally:
            if old is None:
                os.environ.pop("MPCEKF_BOUNDS_SIDE", None)
            else:
                os.environ["MPCEKF_BOUNDS_SIDE"] = old
        outs.append(out)
    for k in ("u", "v", "zk", "zbk"):
        np.testing.assert_array_equal(outs[1][k], outs[0][k], err_msg=k)
    for k in ("ekf", "bigX"):
        np.testing.assert_array_equal(outs[1]["state"][k], outs[0]["state"][k], err_msg=k)
    for t in outs:
        for k in ("bounds", "hild"):
            ms, launches = t["timing"][k]
            assert ms > 0 and launches == 140, (k, ms, launches)


def test_structured_hildreth_edge_paths_match_oracle(oc, M):
    """The fused step's QP solver (rank-2 sweep with its careful and dense fallbacks)
    against the C oracle on structured problems built to reach every path:
    plain problems, a zero G_soc row (Hs[0] = 0) with gamma < 0 (the dense form's
    +inf/NaN alternation), infinite warm starts, a singular E (non-finite X:
    the dense path), and maxIter-bound infeasible duals."""
    rng = np.random.default_rng(31)
    n = 640
    Hv = rng.normal(0, 1e-3, (n, 5))
    He = rng.normal(0, 1e-3, (n, 5))
    Hs = rng.normal(0, 1e-5, (n, 5))
    Hs[:, 0] = 0.0                                            # SOC(k+1) does not see u(k)
    A = rng.normal(0, 1e-2, (n, 2, 2))
    E = A @ A.transpose(0, 2, 1) + 1e-4 * np.eye(2)
    F = rng.normal(0, 1e-2, (n, 2))
    gam = np.abs(rng.normal(0.0, 0.05, (n, 23)))
    lam0 = np.where(rng.random((n, 23)) < 0.3, np.abs(rng.normal(0, 0.5, (n, 23))), 0.0)
    g = np.arange(n) % 8
    gam[g == 1, 18] = -0.01                                   # zero row, gamma < 0
    gam[g == 2, 13:18] = -np.abs(gam[g == 2, 13:18]) - 1e-3   # infeasible eta rows
    lam0[g == 3, 18] = np.inf                                 # warm start from the inf pattern
    E[g == 4] = 0.0                                           # singular E: non-finite X
    F[g == 5] *= 1e3
    DU, lam, ne = M.hildreth_structured(E, F, Hv, He, Hs, gam, lam0)
    assert (ne == 100).any() and (ne < 100).any()
    for i in range(n):
        Mi = M.structured_M(Hv[i], He[i], Hs[i])
        du_r, lam_r, ne_r = oc.hildreth(E[i], F[i], Mi, gam[i], lam0[i], 100)
        assert ne[i] == ne_r, (i, g[i])
        np.testing.assert_array_equal(lam[i], lam_r, err_msg=f"cell {i} group {g[i]}")
        np.testing.assert_array_equal(DU[i], du_r, err_msg=f"cell {i} group {g[i]}")


@pytest.mark.parametrize("Np,Nc", [(5, 2), (20, 10)])
def test_step_diagnostics_match_oracle(rom, oc, M, Np, Nc):
    """Every runMPC.m store per step (mpcekf_step_ex): x_store, zkEst, zkBound and
    mpcData.cost (J_uncon, J_final, norm_DU, viol) against the oracle, bitwise; the
    lock-out cell gives NaN / 0 from its failing step on."""
    n, steps = 24, 40
    soc0, tc = batch_inputs(n, seed=13)
    soc0[3] = 130.0  # lock-out
    ref = oc.run(rom, soc0, tc, steps, nthreads=4, traj=True, Np=Np, Nc=Nc)
    cfg = M.make_config(bounds=True, Np=Np, Nc=Nc)
    names = ("u", "v", "soc", "phise", "nexec", "x", "zk", "zbk", "J_unc", "J_fin", "norm_du", "nviol")
    with M.Context(rom, n, cfg) as ctx:
        ctx.init_cells(soc0, tc)
        out = ctx.step(steps, outputs=names)
        zk_last, zb_last = ctx.get_zk()
    pairs = dict(x="x", zk="zk_traj", zbk="zbk_traj", J_unc="J_unc", J_fin="J_fin", norm_du="norm_du")
    for k, rk in pairs.items():
        _bitwise(out[k], ref[rk], k)
    np.testing.assert_array_equal(out["nviol"], ref["nviol"])
    np.testing.assert_array_equal(out["nexec"], ref["nexec"])
    assert np.isnan(out["zk"][-1, 3]).all() and (out["nviol"][-1, 3] == 0)
    np.testing.assert_array_equal(zk_last, out["zk"][-1])
    np.testing.assert_array_equal(zb_last, out["zbk"][-1])


def test_json_exchanged_rom_is_bit_identical_on_gpu(rom, M, tmp_path):
    """A ROM that went through matlab/mpcekf_export_rom.m's JSON format (ROM.load_json)
    drives the GPU path to bit-identical trajectories: the exchange loses nothing the
    kernels read."""
    p = tmp_path / "rom.json"
    rom.save_json(p)
    q = type(rom).load_json(str(p))
    soc0, tc = batch_inputs(64)
    a = M.runMPC(rom, soc0, tc, 60)
    b = M.runMPC(q, soc0, tc, 60)
    for k in ("u", "v", "soc", "phise", "nexec"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k


def test_temperature_profile_matches_oracle_and_golden(P, oc, M):
    """A temperature per step (runMPC.m:85-92 passes TC to OB_step, iterEKF and
    EKFmatsHandler every call): bitwise against the C oracle over the fused path, and
    within 1e-9 of the numpy restatement's fixture."""
    g = _golden("tprofile4_300")
    rom = P.make_synth_rom()
    steps = g["u"].shape[0]
    out = M.runMPC(rom, g["soc0"], g["tc"], steps, tc_traj=g["tc_traj"])
    ref = oc.run(rom, g["soc0"], g["tc"], steps, nthreads=4, tc_traj=g["tc_traj"])
    for k in ("u", "v", "soc", "phise", "nexec"):
        _bitwise(out[k], ref[k], k)
    np.testing.assert_array_equal(out["status"], g["status"])
    for k in ("u", "v", "soc", "phise"):
        assert _rel(out[k], g[k]).max() <= 1e-9, k


def test_temperature_through_stage_entry_points(rom, M):
    """The stage ABI takes the temperature per call (OB_step(Iapp,Tc,..),
    iterEKF(vk,ik,Tk,..), EKFmatsHandler(..,Tk)): a varying profile through the stage
    calls equals the fused step given the same profile, bit for bit."""
    n, steps = 128, 30
    soc0, tc = batch_inputs(n, seed=17)
    prof = tc[None, :] + 3.0 * np.sin(np.arange(steps)[:, None] / 5.0 + np.arange(n)[None, :] / 9.0)
    fused = M.runMPC(rom, soc0, tc, steps, tc_traj=prof)
    with M.Context(rom, n) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)
        for k in range(steps):
            v = ctx.OB_step(uk, prof[k])
            zk, zb, xind = ctx.iterEKF(v, uk, prof[k])
            lin = ctx.EKFmatsHandler(zk, xind, prof[k])
            uk, ne = ctx.iterMPC(lin, zk[:, -1])
            np.testing.assert_array_equal(v, fused["v"][k])
            np.testing.assert_array_equal(uk, fused["u"][k])
            np.testing.assert_array_equal(ne, fused["nexec"][k])


@pytest.mark.parametrize("Np,Nc", [(5, 2), (20, 10)])
def test_model_blend_matches_oracle_and_golden(P, oc, M, Np, Nc):
    """The model-blend EKF ('MB', iterEKF.m:90-102,125-128,160-176,199-203; initKF.m:47-48,
    111-112) on the GPU: bitwise against the C oracle's ekf_step_mb over the closed loop
    (zk / boundzk and every runMPC.m store included), within 1e-9 of the numpy
    restatement's golden fixture at Np = 5."""
    rom = P.make_synth_rom()
    n, steps = 48, 250
    soc0, tc = batch_inputs(n, seed=23)
    soc0[5] = 130.0                      # thetae < 0 error cell
    cfg = M.make_config(method="MB", bounds=True, Np=Np, Nc=Nc)
    names = ("u", "v", "soc", "phise", "nexec", "x", "zk", "zbk", "J_unc", "J_fin", "norm_du", "nviol")
    with M.Context(rom, n, cfg) as ctx:
        ctx.init_cells(soc0, tc)
        out = ctx.step(steps, outputs=names)
        st = ctx.get_state()
    ref = oc.run(rom, soc0, tc, steps, nthreads=4, traj=True, method="MB", Np=Np, Nc=Nc)
    pairs = dict(u="u", v="v", soc="soc", phise="phise", nexec="nexec", x="x", zk="zk_traj",
                 zbk="zbk_traj", J_unc="J_unc", J_fin="J_fin", norm_du="norm_du", nviol="nviol")
    for k, rk in pairs.items():
        _bitwise(out[k], ref[rk], k)
    np.testing.assert_array_equal(st["status"], ref["status"])
    assert st["status"][5] & 1 and (st["status"][np.arange(n) != 5] == 0).all()
    # the per-model records are never touched by MB (EKFmatsHandler.m:33 reads them)
    assert not st["ekf"][:, :, :5].any()
    assert np.isfinite(st["mb"][st["status"] == 0]).all()
    if (Np, Nc) == (5, 2):
        g = _golden("mb_batch4_200")
        out_g = M.runMPC(rom, g["soc0"], g["tc"], g["u"].shape[0], cfg=M.make_config(method="MB"))
        for k in ("u", "v", "soc", "phise"):
            assert _rel(out_g[k], g[k]).max() <= 1e-9, k
        np.testing.assert_array_equal(out_g["nexec"], g["nexec"])


def test_model_blend_stage_entry_points_match_fused(rom, M):
    n, steps = 64, 20
    soc0, tc = batch_inputs(n, seed=29)
    cfg = M.make_config(method="MB")
    fused = M.runMPC(rom, soc0, tc, steps, cfg=cfg)
    with M.Context(rom, n, cfg) as ctx:
        ctx.init_cells(soc0, tc)
        uk = np.zeros(n)
        for k in range(steps):
            v = ctx.OB_step(uk)
            zk, zb, xind = ctx.iterEKF(v, uk)
            lin = ctx.EKFmatsHandler(zk, xind)
            uk, ne = ctx.iterMPC(lin, zk[:, -1])
            np.testing.assert_array_equal(v, fused["v"][k])
            np.testing.assert_array_equal(uk, fused["u"][k])
            np.testing.assert_array_equal(ne, fused["nexec"][k])


@pytest.mark.parametrize("lookup,block", [("linear", 256), ("linear", 512), ("quintic", 256)])
def test_lane_quad_ekf_kernel_is_exact(P, oc, M, lookup, block):
    """k_ekf4 (iterEKF with a lane quad per cell, MPCEKF_QUAD=1; the 256-thread small-batch
    instantiation spread over the CUs and the 512-thread one; v2 and v3 tables) gives the
    bits of the lane-per-cell k_cell path over a closed loop, state included, and both are
    the C oracle's trajectories."""
    rom = P.make_synth_rom(lookup=lookup)
    n = 700
    soc0, tc = batch_inputs(n, seed=31)
    a = _run_with_env(M, rom, soc0, tc, 120, MPCEKF_QUAD=0)
    b = _run_with_env(M, rom, soc0, tc, 120, MPCEKF_QUAD=1, MPCEKF_EKF4_BLOCK=block)
    ref = oc.run(rom, soc0, tc, 120, nthreads=8)
    for k in ("u", "v", "soc", "phise", "nexec"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        _bitwise(b[k], ref[k], k)
    for k in ("ekf", "bigX", "scal", "lam"):
        np.testing.assert_array_equal(a["state"][k], b["state"][k], err_msg=k)


@pytest.mark.parametrize("Nc,ncon,n", [(10, 100, 96), (3, 17, 64), (1, 9, 64), (2, 40, 64), (7, 61, 48)])
def test_generic_hildreth_any_size_matches_oracle(oc, M, Nc, ncon, n):
    """mpcekf_hildreth (any M) at sizes other than the fused 2 x 23 form, bitwise against
    orc_hildreth: random SPD and non-SPD (LU) E, warm starts, a non-finite M row (the
    dense path) and, at 10 x 100, the constraintsMPC.m shape of configs[4]."""
    rng = np.random.default_rng(100 + Nc * 7 + ncon)
    E = np.empty((n, Nc, Nc))
    for i in range(n):
        A = rng.normal(0, 1, (Nc, Nc))
        E[i] = A @ A.T + 0.3 * np.eye(Nc)
        if i % 11 == 5:  # symmetric, not positive definite: MATLAB's \\ falls back to LU
            E[i] -= (np.linalg.eigvalsh(E[i]).max() * 0.6) * np.eye(Nc)
        E[i] = (E[i] + E[i].T) / 2
    F = rng.normal(0, 1, (n, Nc))
    Mm = rng.normal(0, 1, (n, ncon, Nc))
    if (Nc, ncon) == (10, 100):
        for i in range(0, n, 2):  # [Cu; -Cu; I; -I; G_v; -G_e; G_soc] with Toeplitz blocks
            cu = np.tril(np.ones((Nc, Nc)))
            blocks = []
            for sgn in (1, -1, 1):
                h = rng.normal(0, 1e-2, 20)
                blocks.append(sgn * np.array([[h[r - k] if k <= r else 0.0 for k in range(Nc)] for r in range(20)]))
            Mm[i] = np.vstack([cu, -cu, np.eye(Nc), -np.eye(Nc)] + blocks)
    Mm[3, 1, 0] = np.inf  # the dense path (non-finite M)
    g = rng.normal(0.2, 1, (n, ncon))
    lam0 = np.abs(rng.normal(0, 0.05, (n, ncon)))
    DU, lam, ne = M.hildreth(E, F, Mm, g, lam0, 100)
    for i in range(n):
        d2, l2, k2 = oc.hildreth(E[i], F[i], Mm[i], g[i], lam0[i], 100)
        assert ne[i] == k2, i
        _bitwise(DU[i], d2, f"DU[{i}]")
        _bitwise(lam[i], l2, f"lambda[{i}]")
    assert (ne == 100).any() and (ne < 100).any()


def test_graph_replay_is_exact(rom, oc, M):
    """mpcekf_set_graph: repeated call shapes replayed from captured hipGraphs give the
    bits of direct launches (calls of 1 and 5 steps, shapes alternating, host outputs),
    and the concatenated trajectory is the C oracle's."""
    n = 192
    soc0, tc = batch_inputs(n, seed=21)
    runs = []
    for graph in (False, True):
        with M.Context(rom, n) as ctx:
            ctx.init_cells(soc0, tc)
            ctx.set_graph(graph)
            got = []
            for call in range(30):
                ns = 1 if call % 3 else 5
                out = ctx.step(ns, outputs=("u", "v", "soc", "phise", "nexec"))
                got.append(out)
            st = ctx.get_state()
            runs.append((got, st))
    (a, sa), (b, sb) = runs
    for x, y in zip(a, b):
        for k in x:
            _bitwise(x[k], y[k], k)
    for k in ("bigX", "ekf", "scal", "lam", "status"):
        _bitwise(sa[k], sb[k], k)
    ref = oc.run(rom, soc0, tc, sum(o["u"].shape[0] for o in b), nthreads=4)
    for k in ("u", "v", "soc", "phise", "nexec"):
        _bitwise(np.concatenate([o[k] for o in b]), ref[k], k)


@pytest.mark.parametrize("Np,Nc", [(5, 2), (20, 10)])
def test_graph_replay_temperature_profile_and_diagnostics(oc, M, P, Np, Nc):
    """Graph replay with a temperature profile per call (the profile buffer is part of the
    captured shape, its contents change every call), the cost log and the stability
    diagnostics, at both horizons: replayed calls equal direct launches and the C
    oracle's trajectory with the same profile."""
    rom = P.make_synth_rom()
    n, calls, ns = 64, 8, 3
    soc0, tc = batch_inputs(n, seed=61)
    prof = tc[None, :] + 2.5 * np.sin(np.arange(calls * ns)[:, None] / 4.0 + np.arange(n)[None, :] / 7.0)
    names = ("u", "v", "soc", "phise", "nexec", "J_unc", "J_fin", "norm_du", "nviol", "poles", "sv")
    runs = []
    for graph in (False, True):
        with M.Context(rom, n, M.make_config(Np=Np, Nc=Nc)) as ctx:
            ctx.init_cells(soc0, tc)
            ctx.set_graph(graph)
            runs.append([ctx.step(ns, outputs=names, tc=prof[c * ns:(c + 1) * ns]) for c in range(calls)])
    for x, y in zip(*runs):
        for k in names:
            _bitwise(x[k], y[k], k)
    ref = oc.run(rom, soc0, tc, calls * ns, nthreads=4, traj=True, tc_traj=prof, Np=Np, Nc=Nc)
    for k, rk in dict(u="u", v="v", soc="soc", phise="phise", nexec="nexec", J_unc="J_unc", J_fin="J_fin",
                      norm_du="norm_du", nviol="nviol").items():
        _bitwise(np.concatenate([o[k] for o in runs[1]]), ref[rk], k)
