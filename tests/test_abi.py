"""CPU: the C-ABI library loads and exports every symbol include/mpcekf.h declares
(no compute calls: there is no GPU here), and the host mirror keeps the
reference's function names."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mpcekf.h")).read()
    return sorted(set(re.findall(r"\b(mpcekf_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(P):
    from importlib import import_module
    lib = import_module("mpc-ekf4fastcharge_amd._lib")
    L = lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(lib.EXPORTS)


def test_config_defaults_are_runmpc_values(P):
    from importlib import import_module
    m = import_module("mpc-ekf4fastcharge_amd.mpcekf")
    c = m.make_config()
    assert (c.Np, c.Nc, c.target_soc, c.Crate) == (5, 2, 95.0, 2.0)          # runMPC.m:28-36
    assert (c.u_max, c.du_min, c.du_max, c.v_max, c.phise_min) == (2.0, -50.0, 50.0, 4.1, 0.08)
    assert (c.z_max, c.z_tol, c.max_hild, c.hild_tol) == (0.95, 0.0, 100, 1e-6)
    assert (c.SigmaV, c.SigmaW, list(c.SigmaX0)) == (1e-3, 1e2, [1, 1, 1, 1, 1, 2e6])
    assert (c.use_current, c.use_voltage, c.use_eta, c.max_warn) == (1, 1, 1, 10)


def test_matlab_function_names_present(P):
    from importlib import import_module
    m = import_module("mpc-ekf4fastcharge_amd.mpcekf")
    for name in ("OB_step", "iterEKF", "EKFmatsHandler", "iterMPC"):
        assert callable(getattr(m.Context, name))
    for name in ("predMat", "constraintsMPC", "hildreth", "runMPC"):
        assert callable(getattr(m, name))


def test_last_error_is_empty_string_initially(P):
    from importlib import import_module
    L = import_module("mpc-ekf4fastcharge_amd._lib").load()
    assert isinstance(L.mpcekf_last_error(), bytes)


def test_build_id_is_the_source_hash(P):
    """The library embeds the hash of the sources it was built from (build.py source_hash);
    bench.py attaches PMC traffic only when profiles/pmc_traffic.json was measured on it."""
    from importlib import import_module
    L = import_module("mpc-ekf4fastcharge_amd._lib").load()
    b = import_module("mpc-ekf4fastcharge_amd.build")
    assert L.mpcekf_build_id().decode() == b.source_hash()


# The reference's MATLAB signatures; the drop-in wrappers in
# matlab/dropin must keep them so runMPC.m runs unchanged with that folder first on
# the path.
DROPIN_SIGNATURES = {
    "OB_step": "function [Vcell, obs, cellState] = OB_step(Iapp, Tc, cellState, ROM, initCfg)",
    "iterEKF": "function [zk,boundzk,ekfData,Xind] = iterEKF(vk,ik,Tk,ekfData)",
    "EKFmatsHandler": "function [MPC, xhat] = EKFmatsHandler(ekfData, Xind, zk, Tk)",
    "iterMPC": "function [uk, mpcData] = iterMPC(xk, cellState, mpcData)",
    "hildreth": "function [DU, lambda, nexec] = hildreth(E, F, M, gamma, lambda0, maxIter)",
    "predMat": "function [Phi, G, aug] = predMat(A, B, C, D, Np, Nc)",
    "initKF": "function kfData = initKF(SOC0,T0,SigmaX0,SigmaV,SigmaW,blend,ROMs)",
    "initMPC": "function mpcData = initMPC(SOC0, Np, Nc, targetSOC, opts)",
}


def test_matlab_dropin_wrappers_keep_reference_signatures():
    import re
    d = os.path.join(ROOT, "matlab", "dropin")
    norm = lambda s: re.sub(r"\s+", "", s)
    for name, sig in DROPIN_SIGNATURES.items():
        first = open(os.path.join(d, name + ".m")).readline().strip()
        assert norm(first) == norm(sig), (name, first)


def test_mex_gateway_calls_only_declared_entry_points():
    """matlab/mpcekf_mex.c binds the C-ABI: every mpcekf_* it calls is declared in
    include/mpcekf.h, and every MATLAB-facing stage entry point is reachable from it
    (tests/test_mex_gateway.py drives it through the MEX API test shim)."""
    import re
    src = open(os.path.join(ROOT, "matlab", "mpcekf_mex.c")).read()
    src_code = re.sub(r"/\*.*?\*/", "", src, flags=re.S)  # comments name MATLAB helpers too
    called = set(re.findall(r"\b(mpcekf_[a-z0-9_]+)\s*\(", src_code)) - {"mpcekf_mex"}
    assert called <= set(declared_symbols()), called - set(declared_symbols())
    for sym in ("mpcekf_ctx_create", "mpcekf_init_cells", "mpcekf_step", "mpcekf_plant_step", "mpcekf_ekf_step",
                "mpcekf_linearize", "mpcekf_mpc_step_ex", "mpcekf_hildreth", "mpcekf_predmat", "mpcekf_get_state",
                "mpcekf_set_state", "mpcekf_ctx_destroy", "mpcekf_mpc_diag", "mpcekf_ctx_config"):
        assert sym in called, sym
    drop = " ".join(open(os.path.join(ROOT, "matlab", "dropin", f)).read()
                    for f in os.listdir(os.path.join(ROOT, "matlab", "dropin")))
    cmds = set(re.findall(r"mpcekf_mex\('([a-z_]+)'", drop))
    for c in cmds:
        assert f'"{c}"' in src, c


def test_temperature_argument_rule_is_shared(P):
    """Context.step's tc and oracle_c.run's tc_traj read a temperature argument by one rule
    (ADVICE r03): scalar, a 1-D per-step profile [nsteps], a 1-D per-cell vector [ncells],
    [nsteps, 1], [1, ncells] or the full grid; a 1-D vector of length nsteps == ncells is
    refused as ambiguous instead of being read as per-cell."""
    import numpy as np
    import pytest
    from importlib import import_module
    import oracle_c
    m = import_module("mpc-ekf4fastcharge_amd.mpcekf")
    for f in (m.tc_grid, oracle_c._tc_grid):
        prof = np.arange(5.0)
        np.testing.assert_array_equal(f(prof, 5, 3), np.repeat(prof[:, None], 3, axis=1))   # per step
        cells = np.array([20.0, 21.0, 22.0])
        np.testing.assert_array_equal(f(cells, 5, 3), np.repeat(cells[None, :], 5, axis=0))  # per cell
        np.testing.assert_array_equal(f(25.0, 2, 3), np.full((2, 3), 25.0))
        np.testing.assert_array_equal(f(prof[:, None], 5, 3), np.repeat(prof[:, None], 3, axis=1))
        with pytest.raises(ValueError, match="ambiguous"):
            f(np.arange(4.0), 4, 4)
        with pytest.raises(ValueError):
            f(np.arange(7.0), 5, 3)
