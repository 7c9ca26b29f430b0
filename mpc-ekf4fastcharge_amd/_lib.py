"""ctypes binding of the C-ABI in include/mpcekf.h (libmpcekf.so, built in-tree).

The product path is this library and nothing else: if it is missing the import
fails loudly (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MPCEKF_LIB selects a profiling build (tools/stamps.py); the product path is _build/libmpcekf.so
LIB_PATH = os.environ.get("MPCEKF_LIB") or os.path.join(HERE, "_build", "libmpcekf.so")

MPCEKF_OK = 0
ST_ERROR, ST_LOCKOUT, ST_THETAE_NEG = 1, 2, 4
CF_BOUNDS = 1
LIN_SIZE = 35
NSCAL = 8
MB_SIZE = 42
METHOD_OB, METHOD_MB = 0, 1
S_SOCNAVG, S_SOCPAVG, S_X0, S_SIGMAX0, S_PRIORI, S_UK_1, S_UK, S_VK = range(8)

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class Electrode(C.Structure):
    _fields_ = [("theta0", C.c_double), ("theta100", C.c_double), ("soc0", _dp), ("soc100", _dp),
                ("Uocp", _dp), ("dUocp", _dp), ("k0", _dp), ("Rf", _dp), ("Cdleff", _dp), ("Uocp1", _dp),
                ("Uocp_p", _dp), ("dUocp_p", _dp), ("k0_p", _dp), ("Rf_p", _dp), ("Cdleff_p", _dp),
                ("Uocp1_p", _dp), ("Ea", C.c_double * 5),
                ("nnode", C.c_int32 * 6), ("node", _dp * 6), ("node_p", _dp * 6)]   # ABI v4


class Rom(C.Structure):
    _fields_ = [("nT", C.c_int32), ("nZ", C.c_int32), ("n", C.c_int32), ("nz", C.c_int32),
                ("T_degC", _dp), ("SOC_pct", _dp), ("Ts", C.c_double), ("A", _dp), ("C", _dp),
                ("D", _dp), ("tf_code", _ip), ("tf_xloc", _dp), ("F", C.c_double), ("R", C.c_double),
                ("Q", C.c_double), ("Rc", C.c_double), ("Tref", C.c_double), ("tab_ntheta", C.c_int32),
                ("tab_ntemp", C.c_int32), ("tab_T_K", _dp), ("tab_npoly", C.c_int32), ("neg", Electrode),
                ("pos", Electrode)]


class Config(C.Structure):
    _fields_ = [("Np", C.c_int32), ("Nc", C.c_int32), ("target_soc", C.c_double), ("Crate", C.c_double),
                ("u_max", C.c_double), ("du_min", C.c_double), ("du_max", C.c_double),
                ("v_min", C.c_double), ("v_max", C.c_double), ("phise_min", C.c_double),
                ("z_max", C.c_double), ("z_tol", C.c_double), ("use_current", C.c_int32),
                ("use_voltage", C.c_int32), ("use_eta", C.c_int32), ("max_hild", C.c_int32),
                ("hild_tol", C.c_double), ("SigmaV", C.c_double), ("SigmaW", C.c_double),
                ("SigmaX0", C.c_double * 6), ("max_warn", C.c_int32), ("flags", C.c_int32),
                ("method", C.c_int32)]


class State(C.Structure):
    _fields_ = [("bigX", _dp), ("ekf", _dp), ("scal", _dp), ("lam", _dp), ("warn", _ip), ("status", _ip),
                ("mb", _dp)]


class Traj(C.Structure):
    """mpcekf_traj: per-step output pointers of mpcekf_step_ex (any may be NULL)."""
    _fields_ = [("u", C.c_void_p), ("v", C.c_void_p), ("soc", C.c_void_p), ("phise", C.c_void_p),
                ("nexec", C.c_void_p), ("x", C.c_void_p), ("zk", C.c_void_p), ("zbk", C.c_void_p),
                ("J_unc", C.c_void_p), ("J_fin", C.c_void_p), ("norm_du", C.c_void_p), ("nviol", C.c_void_p),
                ("poles", C.c_void_p), ("sv", C.c_void_p)]


class MpcekfError(RuntimeError):
    pass


EXPORTS = [
    "mpcekf_abi_version", "mpcekf_last_error", "mpcekf_config_defaults", "mpcekf_ctx_create",
    "mpcekf_ctx_destroy", "mpcekf_ctx_info", "mpcekf_ctx_config", "mpcekf_init_cells", "mpcekf_step", "mpcekf_step_ex", "mpcekf_get_zk",
    "mpcekf_plant_step", "mpcekf_ekf_step", "mpcekf_linearize", "mpcekf_mpc_step", "mpcekf_mpc_step_ex", "mpcekf_predmat",
    "mpcekf_constraints", "mpcekf_hildreth", "mpcekf_get_state", "mpcekf_set_state",
    "mpcekf_set_timing", "mpcekf_get_timing", "mpcekf_get_hild_problems", "mpcekf_get_stamps", "mpcekf_hildreth_structured",
    "mpcekf_build_id", "mpcekf_cl_eig", "mpcekf_mpc_diag", "mpcekf_set_graph",
    "mpcekf_dev_alloc", "mpcekf_dev_free", "mpcekf_dev_copy", "mpcekf_dev_copy2d", "mpcekf_sync",
    "mpcekf_get_scalars", "mpcekf_lin_fields",
    # the _async stage twins (include/mpcekf.h)
    "mpcekf_plant_step_async", "mpcekf_ekf_step_async", "mpcekf_linearize_async", "mpcekf_lin_fields_async",
    "mpcekf_mpc_step_async", "mpcekf_mpc_step_ex_async", "mpcekf_mpc_diag_async", "mpcekf_get_scalars_async",
]

COPY_H2D, COPY_D2H, COPY_D2D = 0, 1, 2
ABI_VERSION = 4   # include/mpcekf.h MPCEKF_ABI_VERSION

_lib = None


def load():
    """Load libmpcekf.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpcekfError(f"{LIB_PATH} not found: run __graft_entry__.build() (hipcc gfx950)")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.mpcekf_abi_version.restype = C.c_int
    L.mpcekf_last_error.restype = C.c_char_p
    L.mpcekf_build_id.restype = C.c_char_p
    L.mpcekf_config_defaults.argtypes = [C.POINTER(Config)]
    L.mpcekf_config_defaults.restype = None
    L.mpcekf_ctx_create.argtypes = [C.POINTER(Rom), C.POINTER(Config), C.c_int, C.c_int64, C.POINTER(vp)]
    L.mpcekf_ctx_destroy.argtypes = [vp]
    L.mpcekf_ctx_info.argtypes = [vp, C.POINTER(C.c_int64), _ip, _ip, _ip]
    L.mpcekf_ctx_config.argtypes = [vp, C.POINTER(Config)]
    L.mpcekf_init_cells.argtypes = [vp, _dp, _dp]
    L.mpcekf_step.argtypes = [vp, C.c_int32, vp, vp, vp, vp, vp, vp, C.c_int32]
    L.mpcekf_step_ex.argtypes = [vp, C.c_int32, vp, C.POINTER(Traj), C.c_int32]
    L.mpcekf_get_zk.argtypes = [vp, _dp, _dp]
    L.mpcekf_plant_step.argtypes = [vp, _dp, _dp, _dp]
    L.mpcekf_ekf_step.argtypes = [vp, _dp, _dp, _dp, _dp, _dp, _ip, _dp]
    L.mpcekf_linearize.argtypes = [vp, _dp, _ip, _dp, _dp, _dp]
    L.mpcekf_mpc_step.argtypes = [vp, _dp, _dp, _dp, _ip]
    L.mpcekf_mpc_step_ex.argtypes = [vp, _dp, _dp, _dp, _ip, _dp, _dp, _dp, _ip]
    L.mpcekf_predmat.argtypes = [C.c_int, C.c_int64, C.c_int32, C.c_int32, _dp, _dp, _dp, _dp, _dp]
    L.mpcekf_constraints.argtypes = [C.c_int, C.POINTER(Config), C.c_double, C.c_int64, _dp, _dp, _dp,
                                     _dp, _dp]
    L.mpcekf_hildreth.argtypes = [C.c_int, C.c_int64, C.c_int32, C.c_int32, _dp, _dp, _dp, _dp, _dp,
                                  C.c_int32, C.c_double, _dp, _ip]
    L.mpcekf_get_state.argtypes = [vp, C.POINTER(State)]
    L.mpcekf_set_state.argtypes = [vp, C.POINTER(State)]
    L.mpcekf_set_timing.argtypes = [vp, C.c_int32]
    L.mpcekf_set_graph.argtypes = [vp, C.c_int32]
    L.mpcekf_get_timing.argtypes = [vp, _dp, C.POINTER(C.c_int64)]
    L.mpcekf_get_hild_problems.argtypes = [vp, _dp, _ip]
    L.mpcekf_get_stamps.argtypes = [vp, C.POINTER(C.c_int64), _ip]
    L.mpcekf_cl_eig.argtypes = [C.c_int32, _dp, _dp, _dp, _dp]
    L.mpcekf_mpc_diag.argtypes = [vp, _dp, _dp, _dp, _dp]
    L.mpcekf_hildreth_structured.argtypes = [C.c_int, C.c_int64, _dp, _dp, _dp, _dp, _dp, _dp, _dp, C.c_int32,
                                             C.c_double, _dp, _ip]
    L.mpcekf_dev_alloc.argtypes = [C.c_int, C.c_int64, C.POINTER(vp)]
    L.mpcekf_dev_free.argtypes = [vp]
    L.mpcekf_dev_copy.argtypes = [vp, vp, C.c_int64, C.c_int32]
    L.mpcekf_dev_copy2d.argtypes = [vp, C.c_int64, vp, C.c_int64, C.c_int64, C.c_int64, C.c_int32]
    L.mpcekf_sync.argtypes = [vp]
    L.mpcekf_get_scalars.argtypes = [vp, _ip, C.c_int32, _dp, _ip, _ip]
    L.mpcekf_lin_fields.argtypes = [vp, _ip, C.c_int32, _dp, _dp]
    for nm in ("plant_step", "ekf_step", "linearize", "lin_fields", "mpc_step", "mpc_step_ex", "mpc_diag",
               "get_scalars"):   # the _async twins take the synchronous call's arguments
        getattr(L, f"mpcekf_{nm}_async").argtypes = getattr(L, f"mpcekf_{nm}").argtypes
    for nm in EXPORTS:
        if nm not in ("mpcekf_abi_version", "mpcekf_last_error", "mpcekf_config_defaults", "mpcekf_build_id"):
            getattr(L, nm).restype = C.c_int
    if L.mpcekf_abi_version() != ABI_VERSION:
        raise MpcekfError("ABI version mismatch")
    _lib = L
    return L


def check(rc):
    if rc != MPCEKF_OK:
        raise MpcekfError(f"mpcekf error {rc}: {_lib.mpcekf_last_error().decode()}")


def dptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


def iptr(a):
    return a.ctypes.data_as(_ip) if a is not None else None
