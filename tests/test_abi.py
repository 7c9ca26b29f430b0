"""CPU: the C-ABI library loads and exports every symbol include/mpcekf.h declares
(no compute calls: there is no GPU here), and the host mirror keeps the
reference's function names."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mpcekf.h")).read()
    return sorted(set(re.findall(r"\b(mpcekf_[a-z_]+)\s*\(", src)))


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
