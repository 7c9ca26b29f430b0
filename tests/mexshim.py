"""ctypes driver of the MEX gateway (matlab/mpcekf_mex.c) built against the MEX API test
shim (tests/mex: mex.h, matrix.h, mexshim.c -- not MATLAB).

``mex(cmd, *args, nargout=1)`` calls mexFunction the way MATLAB would: every argument is
converted to an mxArray with MATLAB's class and column-major layout (numpy arrays keep
their shape; Python floats/ints become 1 x 1 doubles; dicts become 1 x 1 structs; str a
char row), and the outputs come back as numpy arrays of MATLAB's shape (Fortran order)
or dicts.  A MEX error raises :class:`MexError` with the gateway's message.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("MEXSHIM_LIB") or os.path.join(HERE, "mex", "_build", "libmpcekf_mexshim.so")

DOUBLE, INT32, UINT64, STRUCT, CHAR = 6, 12, 15, 2, 4
_NP = {DOUBLE: np.float64, INT32: np.int32, UINT64: np.uint64, 7: np.float32, 8: np.int8, 9: np.uint8,
       10: np.int16, 11: np.uint16, 13: np.uint32, 14: np.int64, 3: np.uint8}
_CLS = {np.dtype(v): k for k, v in _NP.items() if k != 3}


class MexError(RuntimeError):
    pass


_lib = None


def build():
    import subprocess
    if not os.environ.get("MEXSHIM_LIB"):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "mex")], check=True)


def load():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.shim_numeric.restype = vp
        L.shim_numeric.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_size_t), vp, C.c_int]
        L.shim_string.restype = vp
        L.shim_string.argtypes = [C.c_char_p]
        L.shim_struct.restype = vp
        L.shim_set_field.argtypes = [vp, C.c_char_p, vp]
        L.shim_get_field.restype = vp
        L.shim_get_field.argtypes = [vp, C.c_char_p]
        L.shim_nfields.argtypes = [vp]
        L.shim_field_name.restype = C.c_char_p
        L.shim_field_name.argtypes = [vp, C.c_int]
        L.shim_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_size_t),
                                C.POINTER(C.c_void_p)]
        L.shim_destroy.argtypes = [vp]
        L.shim_last_error.restype = C.c_char_p
        L.shim_call.argtypes = [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp)]
        L.shim_clear_mex.restype = C.c_int
        _lib = L
    return _lib


def to_mx(x):
    """Python / numpy value -> mxArray pointer (caller destroys)."""
    L = load()
    if isinstance(x, dict):
        s = L.shim_struct()
        for k, v in x.items():
            L.shim_set_field(s, k.encode(), to_mx(v))
        return s
    if isinstance(x, str):
        return L.shim_string(x.encode())
    if isinstance(x, complex) or (isinstance(x, np.ndarray) and np.iscomplexobj(x)):
        a = np.asarray(x, dtype=np.complex128)
        a2 = np.atleast_2d(a) if a.ndim < 2 else a
        f = np.asfortranarray(a2)
        inter = np.empty(f.size * 2)
        inter[0::2] = f.real.ravel(order="F")
        inter[1::2] = f.imag.ravel(order="F")
        dims = (C.c_size_t * a2.ndim)(*a2.shape)
        return L.shim_numeric(DOUBLE, a2.ndim, dims, inter.ctypes.data_as(C.c_void_p), 1)
    a = np.asarray(x)
    if a.dtype == np.bool_:
        a = a.astype(np.float64)
    if a.dtype.kind in "iu" and not isinstance(x, np.ndarray):
        a = a.astype(np.float64)  # a Python int is a MATLAB double
    if a.dtype == np.float64 or a.dtype.kind == "f" and a.dtype != np.float32:
        a = a.astype(np.float64)
    if a.ndim < 2:
        a = a.reshape((1, -1)) if a.ndim == 1 else a.reshape((1, 1))
    cls = _CLS[a.dtype]
    flat = np.ascontiguousarray(a.ravel(order="F"))
    dims = (C.c_size_t * a.ndim)(*a.shape)
    return L.shim_numeric(cls, a.ndim, dims, flat.ctypes.data_as(C.c_void_p), 0)


def from_mx(p):
    """mxArray pointer -> numpy array (MATLAB shape) or dict; does not destroy."""
    L = load()
    cls, cplx = C.c_int(), C.c_int()
    dims = (C.c_size_t * 8)()
    data = C.c_void_p()
    nd = L.shim_info(p, C.byref(cls), C.byref(cplx), dims, C.byref(data))
    shape = tuple(dims[i] for i in range(nd))
    if cls.value == STRUCT:
        return {L.shim_field_name(p, i).decode(): from_mx(L.shim_get_field(p, L.shim_field_name(p, i)))
                for i in range(L.shim_nfields(p))}
    n = int(np.prod(shape))
    if cls.value == CHAR:
        return C.string_at(data, n).decode()
    dt = np.dtype(_NP[cls.value])
    k = n * (2 if cplx.value else 1)
    buf = np.ctypeslib.as_array(C.cast(data, C.POINTER(C.c_byte)), shape=(k * dt.itemsize,)).copy() if k else \
        np.zeros(0, np.byte)
    flat = buf.view(dt)
    if cplx.value:
        flat = flat[0::2] + 1j * flat[1::2]
    return flat.reshape(shape, order="F")


def mex(cmd, *args, nargout=1):
    """[out1, ..., outN] = mpcekf_mex(cmd, args...) through the shim.  Checks that the
    gateway writes no output beyond max(nargout, 1) (MATLAB's plhs is that long)."""
    L = load()
    ins = [to_mx(cmd)] + [to_mx(a) for a in args]
    prhs = (C.c_void_p * len(ins))(*ins)
    keep = max(nargout, 1)
    guard = 8
    plhs = (C.c_void_p * (keep + guard))()
    try:
        rc = L.shim_call(nargout, plhs, len(ins), prhs)
        if any(plhs[keep + i] for i in range(guard)):
            raise AssertionError("gateway wrote outputs beyond max(nargout, 1)")
        if rc:
            raise MexError(L.shim_last_error().decode())
        outs = [from_mx(plhs[i]) if plhs[i] else None for i in range(nargout)]
        for i in range(keep):
            if plhs[i]:
                L.shim_destroy(plhs[i])
    finally:
        for p in ins:
            L.shim_destroy(p)
    return outs[0] if nargout == 1 else tuple(outs)


def clear_mex():
    """MATLAB's `clear mex`: runs the gateway's mexAtExit function; True if one was set."""
    return bool(load().shim_clear_mex())


def rom_struct(rom):
    """The R struct mpcekf_rom_struct.m builds (what 'create' takes), from a rom.ROM:
    A nT x nZ x (n+1), C nT x nZ x nz x (n+1), D nT x nZ x nz, electrode tables
    ntemp x ntheta -- MATLAB's shapes, column-major in the mxArrays."""
    from importlib import import_module
    codes = import_module("mpc-ekf4fastcharge_amd.rom").TF_CODE

    def el(e):
        return dict(theta0=float(e.theta0), theta100=float(e.theta100), soc0=np.asarray(e.soc0, float),
                    soc100=np.asarray(e.soc100, float), Uocp=np.asarray(e.Uocp, float),
                    dUocp=np.asarray(e.dUocp, float), k0=np.asarray(e.k0, float), Rf=np.asarray(e.Rf, float),
                    Cdleff=np.asarray(e.Cdleff, float), Uocp1=np.asarray(e.Uocp1, float))

    def el3(e):   # ABI v3: theta polynomials and Arrhenius energies (mpcekf_rom_struct.m's poly / Ea)
        d = el(e)
        if e.poly:
            d["poly"] = {k: np.asarray(v, float) for k, v in e.poly.items()}
        if e.Ea:
            d["Ea"] = np.array([float(e.Ea.get(k, 0.0)) for k in ("Uocp", "dUocp", "k0", "Rf", "Cdleff")])
        if e.nodes:   # ABI v4 (mpcekf_build_tables.m's nodes): p padded to the poly tables' order
            def pad(c):
                c = np.asarray(c, float)
                return np.concatenate([c, np.zeros(c.shape[:-1] + (rom.npoly - c.shape[-1],))], -1)
            d["nodes"] = {k: {"x": np.asarray(x, float), "p": pad(c)} for k, (x, c) in e.nodes.items()}
        return d
    el_ = el3
    return dict(T_degC=np.asarray(rom.T_degC, float), SOC_pct=np.asarray(rom.SOC_pct, float), Ts=float(rom.Ts),
                A=np.asarray(rom.A, float), C=np.asarray(rom.C, float), D=np.asarray(rom.D, float),
                tf_code=np.array([codes[nm] for nm in rom.names], np.int32), xloc=np.asarray(rom.xloc, float),
                F=float(rom.F), R=float(rom.R), Q=float(rom.Q), Rc=float(rom.Rc), Tref=float(rom.Tref),
                tab_T_K=np.atleast_1d(np.asarray(rom.tab_T_K, float)), neg=el_(rom.neg), pos=el_(rom.pos))


def default_table_temps(T_set, TC, nmax=8):
    """matlab/mpcekf_rom_struct.m's default TdegC, restated: the ROM set-point temperatures
    and the distinct simulation temperatures TC (only their span when they would not fit
    the nmax slots), evenly nmax points when the set-points + span still do not, guard
    points 10 degC beyond when 2 slots are free, then spare slots halve the widest
    intervals (the first widest on ties, as MATLAB's max)."""
    Ts = [float(t) for t in np.ravel(T_set)]
    TCu = sorted(set(float(t) for t in np.ravel(TC)))
    if len(set(Ts) | set(TCu)) > nmax:
        TCu = sorted({min(TCu), max(TCu)})
    T = sorted(set(Ts) | set(TCu))
    if len(T) > nmax:
        T = list(np.linspace(min(T), max(T), nmax))
    if len(T) + 2 <= nmax:
        T = sorted(set([T[0] - 10] + T + [T[-1] + 10]))
    while len(T) < nmax:
        d = np.diff(T)
        k = int(np.argmax(d))
        T = T[:k + 1] + [(T[k] + T[k + 1]) / 2] + T[k + 1:]
    return np.array(T)
