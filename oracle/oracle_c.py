"""ctypes front-end of oracle/mpcekf_oracle.c -- TEST INFRASTRUCTURE ONLY.

PARITY UNPINNED (see oracle_np.py).  Used by tests/ as the checker of the HIP
kernels and by bench.py's ``cpu_baseline`` leg (kind "port").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: the sanitizer build (tools/sanitize.sh) in place of the default one
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "_build", "liboracle.so")

TF_CODES = {n: i for i, n in enumerate([
    "negIfdl", "posIfdl", "negIf", "posIf", "negIdl", "posIdl", "negPhis", "posPhis",
    "negPhise", "posPhise", "negThetass", "posThetass", "negPhie", "sepPhie", "posPhie",
    "negThetae", "sepThetae", "posThetae"])}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class _Electrode(C.Structure):
    _fields_ = [("theta0", C.c_double), ("theta100", C.c_double), ("soc0", _dp), ("soc100", _dp),
                ("Uocp", _dp), ("dUocp", _dp), ("k0", _dp), ("Rf", _dp), ("Cdleff", _dp), ("Uocp1", _dp),
                ("Uocp_p", _dp), ("dUocp_p", _dp), ("k0_p", _dp), ("Rf_p", _dp), ("Cdleff_p", _dp),
                ("Uocp1_p", _dp), ("Ea", C.c_double * 5), ("tconst", C.c_int),
                ("nnode", C.c_int * 6), ("node", _dp * 6), ("node_p", _dp * 6)]   # ABI v4


EL_FNS = ("Uocp", "dUocp", "k0", "Rf", "Cdleff")   # orc_electrode.Ea order (EF_*)


def poly6(c):
    """v3 theta polynomials padded to the 6 coefficients the C oracle and the library
    evaluate (a cubic's c4 = c5 = 0)."""
    c = np.asarray(c, dtype=np.float64)
    if c.shape[-1] == 6:
        return c
    pad = np.zeros(c.shape[:-1] + (6 - c.shape[-1],))
    return np.concatenate([c, pad], axis=-1)


class _Rom(C.Structure):
    _fields_ = [("nT", C.c_int), ("nZ", C.c_int), ("n", C.c_int), ("nz", C.c_int),
                ("T_degC", _dp), ("SOC_pct", _dp), ("Ts", C.c_double), ("A", _dp), ("C", _dp),
                ("D", _dp), ("tf", _ip), ("xloc", _dp), ("F", C.c_double), ("R", C.c_double),
                ("Q", C.c_double), ("Rc", C.c_double), ("Tref", C.c_double),
                ("ntheta", C.c_int), ("ntemp", C.c_int), ("TK", _dp),
                ("neg", _Electrode), ("pos", _Electrode)]


class _Cfg(C.Structure):
    _fields_ = [("Np", C.c_int), ("Nc", C.c_int), ("ref", C.c_double), ("u_max", C.c_double),
                ("Crate", C.c_double), ("du_min", C.c_double), ("du_max", C.c_double),
                ("v_max", C.c_double), ("phise_min", C.c_double), ("z_max", C.c_double),
                ("z_tol", C.c_double), ("use_cur", C.c_int), ("use_v", C.c_int),
                ("use_eta", C.c_int), ("maxHild", C.c_int), ("hild_tol", C.c_double),
                ("SigmaV", C.c_double), ("SigmaW", C.c_double), ("SigmaX0", C.c_double * 6),
                ("max_warn", C.c_int), ("method", C.c_int)]


def build(quiet=True):
    if os.environ.get("ORACLE_LIB"):  # a prebuilt variant (tools/sanitize.sh)
        return
    subprocess.run(["make", "-s", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


_lib = None


def _host_has_fma():
    try:
        with open("/proc/cpuinfo") as f:
            return any(line.startswith("flags") and " fma " in line + " " for line in f)
    except OSError:
        return True


def lib():
    global _lib
    if _lib is None:
        if not _host_has_fma():
            raise RuntimeError("the C oracle is built with -mfma (FMA3); this host CPU lacks it")
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_run.restype = C.c_int
        L.orc_run.argtypes = [C.POINTER(_Rom), C.POINTER(_Cfg), C.c_int, _dp, _dp, C.c_int,
                              _dp, _dp, _dp, _dp, _ip, _ip, _dp, _dp, C.c_int]
        L.orc_predmat.argtypes = [_dp, _dp, C.c_double, C.c_int, C.c_int, _dp, _dp]
        L.orc_hildreth.restype = C.c_int
        L.orc_hildreth.argtypes = [C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp, C.c_int, C.c_double, _dp]
        L.orc_run_traj.restype = C.c_int
        L.orc_run_traj.argtypes = [C.POINTER(_Rom), C.POINTER(_Cfg), C.c_int, _dp, _dp, C.c_int,
                                   _dp, _dp, _dp, _dp, _ip, _ip, _dp, _dp, C.POINTER(_Traj), C.c_int]
        L.orc_mpc_lin.restype = C.c_int
        L.orc_mpc_lin.argtypes = [C.POINTER(_Rom), C.POINTER(_Cfg), C.c_int, _dp, _dp, _dp, _dp, _dp, _ip]
        L.orc_sigma_min.restype = C.c_double
        L.orc_sigma_min.argtypes = [C.c_int, _dp]
        L.orc_meas_cov.argtypes = [_dp, _dp, C.c_double, C.c_int]
        L.orc_jacobi.argtypes = [C.c_int, _dp, _dp, _dp]
        L.orc_exp.restype = C.c_double      # the v3 Arrhenius factor's defined exp
        L.orc_exp.argtypes = [C.c_double]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_dp)


class PackedRom:
    """Keeps the numpy buffers alive for the lifetime of the struct."""

    def __init__(self, rom):
        self.keep = []

        def arr(x, dt=np.float64):
            a = np.ascontiguousarray(x, dtype=dt)
            self.keep.append(a)
            return a

        r = _Rom()
        r.nT, r.nZ, r.n, r.nz = rom.nT, rom.nZ, rom.n, rom.nz
        r.T_degC = _p(arr(rom.T_degC))
        r.SOC_pct = _p(arr(rom.SOC_pct))
        r.Ts = rom.Ts
        r.A = _p(arr(rom.A))
        r.C = _p(arr(rom.C))
        r.D = _p(arr(rom.D))
        r.tf = arr([TF_CODES[n] for n in rom.names], np.int32).ctypes.data_as(_ip)
        r.xloc = _p(arr(rom.xloc))
        r.F, r.R, r.Q, r.Rc, r.Tref = rom.F, rom.R, rom.Q, rom.Rc, rom.Tref
        r.ntheta, r.ntemp = rom.ntheta, rom.ntemp
        r.TK = _p(arr(np.atleast_1d(rom.tab_T_K)))
        for side in ("neg", "pos"):
            e = getattr(rom, side)
            s = getattr(r, side)
            s.theta0, s.theta100 = e.theta0, e.theta100
            for k in ("soc0", "soc100", "Uocp", "dUocp", "k0", "Rf", "Cdleff", "Uocp1"):
                setattr(s, k, _p(arr(getattr(e, k))))
            nd = e.nodes or {}
            for k in EL_FNS + ("Uocp1",):   # ABI v3 polynomials (NULL: linear tables)
                setattr(s, k + "_p", _p(arr(poly6(e.poly[k]))) if e.poly and k in e.poly else _dp())
            for i, k in enumerate(EL_FNS):
                s.Ea[i] = float((e.Ea or {}).get(k, 0.0))
                # rows all equal (an exact Arrhenius function): row 0 blended with itself (the library's one path)
                rows = np.asarray(nd[k][1]) if k in nd else (np.asarray(e.poly[k]) if e.poly else None)
                if rows is not None and rows.shape[0] > 1 and all(np.array_equal(rows[0], rows[j])
                                                                  for j in range(1, rows.shape[0])):
                    s.tconst |= 1 << i
            for i, k in enumerate(EL_FNS + ("Uocp1",)):   # ABI v4 node tables
                if k in nd:
                    s.nnode[i] = int(np.asarray(nd[k][0]).size)
                    s.node[i] = _p(arr(nd[k][0]))
                    s.node_p[i] = _p(arr(poly6(nd[k][1])))
        self.s = r


DEFAULTS = dict(Np=5, Nc=2, ref=95.0, u_max=2.0, Crate=2.0, du_min=-50.0, du_max=50.0, v_max=4.1,
                phise_min=0.08, z_max=0.95, z_tol=0.0, constraints=(1, 1, 1), maxHild=100,
                hild_tol=1e-6, SigmaV=1e-3, SigmaW=1e2, SigmaX0=(1, 1, 1, 1, 1, 2e6), max_warn=10,
                method="OB")


def make_cfg(**kw):
    d = dict(DEFAULTS)
    d.update(kw)
    c = _Cfg()
    c.Np, c.Nc = d["Np"], d["Nc"]
    for k in ("ref", "u_max", "Crate", "du_min", "du_max", "v_max", "phise_min", "z_max", "z_tol",
              "hild_tol", "SigmaV", "SigmaW"):
        setattr(c, k, float(d[k]))
    c.use_cur, c.use_v, c.use_eta = (int(x) for x in d["constraints"])
    c.maxHild = d["maxHild"]
    c.max_warn = d["max_warn"]
    c.method = {"OB": 0, "OUTB": 0, "MB": 1, "MDLB": 1}[str(d["method"]).upper()]   # initKF.m:44-49
    for i in range(6):
        c.SigmaX0[i] = float(d["SigmaX0"][i])
    return c


class _Traj(C.Structure):
    _fields_ = [("x", _dp), ("zk", _dp), ("zbk", _dp), ("J_unc", _dp), ("J_fin", _dp), ("norm_du", _dp),
                ("nviol", _ip), ("tc", _dp)]


def _tc_grid(tc, nsteps, n):
    """[nsteps, n] per-step temperatures: scalar, 1-D per step [nsteps] or per cell [n]
    (refused when nsteps == n), [nsteps, 1], [1, n] or the full grid (the library's
    mpcekf.tc_grid rule, restated here so the checker imports nothing of the product)."""
    a = np.asarray(tc, dtype=np.float64)
    if a.ndim == 1 and a.size != 1:
        if a.size == nsteps and a.size == n:
            raise ValueError("tc_traj: 1-D vector with nsteps == ncells is ambiguous")
        if a.size == nsteps:
            a = a.reshape(nsteps, 1)
        elif a.size == n:
            a = a.reshape(1, n)
        else:
            raise ValueError("tc_traj: length is neither nsteps nor ncells")
    return np.ascontiguousarray(np.broadcast_to(a, (nsteps, n)))


def run(rom, soc0, tc, nsteps, nthreads=0, want_zk=False, traj=False, tc_traj=None, **cfg):
    """Batched closed loop on the CPU. Returns dict of [nsteps, ncells] arrays.

    traj=True adds the per-step diagnostics of runMPC.m:106-111 / mpcData.cost:
    x [nsteps, n, 6], zk_traj / zbk_traj [nsteps, n, nz+2], J_unc, J_fin, norm_du, nviol.
    tc_traj [nsteps, ncells] (degC): the temperature of each step (tc is the initial one)."""
    soc0 = np.ascontiguousarray(soc0, dtype=np.float64)
    tc = np.ascontiguousarray(tc, dtype=np.float64)
    n = soc0.shape[0]
    pr = PackedRom(rom)
    c = make_cfg(**cfg)
    out = {k: np.zeros((nsteps, n)) for k in ("u", "v", "soc", "phise")}
    out["nexec"] = np.zeros((nsteps, n), dtype=np.int32)
    out["status"] = np.zeros(n, dtype=np.int32)
    zk = np.zeros((n, rom.nz + 2)) if want_zk else None
    zbk = np.zeros((n, rom.nz + 2)) if want_zk else None
    tr = None
    tcs = None
    if tc_traj is not None:
        tcs = _tc_grid(tc_traj, nsteps, n)
        tr = _Traj()
        tr.tc = _p(tcs)
    if traj:
        out["x"] = np.zeros((nsteps, n, 6))
        out["zk_traj"] = np.zeros((nsteps, n, rom.nz + 2))
        out["zbk_traj"] = np.zeros((nsteps, n, rom.nz + 2))
        for k in ("J_unc", "J_fin", "norm_du"):
            out[k] = np.zeros((nsteps, n))
        out["nviol"] = np.zeros((nsteps, n), dtype=np.int32)
        tr = _Traj(_p(out["x"]), _p(out["zk_traj"]), _p(out["zbk_traj"]), _p(out["J_unc"]), _p(out["J_fin"]),
                   _p(out["norm_du"]), out["nviol"].ctypes.data_as(_ip), _p(tcs) if tcs is not None else None)
    rc = lib().orc_run_traj(C.byref(pr.s), C.byref(c), n, _p(soc0), _p(tc), nsteps, _p(out["u"]),
                            _p(out["v"]), _p(out["soc"]), _p(out["phise"]),
                            out["nexec"].ctypes.data_as(_ip), out["status"].ctypes.data_as(_ip),
                            _p(zk) if want_zk else None, _p(zbk) if want_zk else None,
                            C.byref(tr) if tr is not None else None, nthreads)
    if rc:
        raise RuntimeError(f"orc_run failed: {rc}")
    if want_zk:
        out["zk"], out["zbk"] = zk, zbk
    return out


def mpc_lin(rom, lin, soc_k1, uk_1, lam, **cfg):
    """iterMPC.m on given linearisation records [n, 35]; uk_1 [n] and lam [n, ncon] are the
    mpcData state (copied).  Returns uk, nexec, uk_1 after, lam after."""
    lin = np.ascontiguousarray(lin, dtype=np.float64)
    n = lin.shape[0]
    pr = PackedRom(rom)
    c = make_cfg(**cfg)
    u1 = np.array(uk_1, dtype=np.float64)
    lm = np.array(lam, dtype=np.float64, order="C")
    uk = np.empty(n)
    ne = np.empty(n, dtype=np.int32)
    rc = lib().orc_mpc_lin(C.byref(pr.s), C.byref(c), n, _p(lin), _p(np.ascontiguousarray(soc_k1, dtype=np.float64)),
                           _p(u1), _p(lm), _p(uk), ne.ctypes.data_as(_ip))
    if rc:
        raise RuntimeError(f"orc_mpc_lin failed: {rc}")
    return uk, ne, u1, lm


def predmat(a, Cr, D, Np, Nc):
    Phi = np.zeros((Np, 7))
    G = np.zeros((Np, Nc))
    lib().orc_predmat(_p(np.ascontiguousarray(a, float)), _p(np.ascontiguousarray(Cr, float)),
                      float(D), Np, Nc, _p(Phi), _p(G))
    return Phi, G


def hildreth(E, F, M, gamma, lam0, maxIter=100, tol=1e-6):
    E = np.ascontiguousarray(E, float)
    M = np.ascontiguousarray(M, float)
    lam = np.array(lam0, dtype=float)
    DU = np.zeros(E.shape[0])
    it = lib().orc_hildreth(E.shape[0], M.shape[0], _p(E), _p(np.ascontiguousarray(F, float)), _p(M),
                            _p(np.ascontiguousarray(gamma, float)), _p(lam), maxIter, tol, _p(DU))
    return DU, lam, it


def sigma_min(G):
    G = np.ascontiguousarray(G, float)
    return lib().orc_sigma_min(G.shape[0], _p(G))
