"""Host-side mirror of the reference's operator interface, over the C-ABI.

The reference exposes MATLAB functions called by name from runMPC.m; this
module keeps those names and argument meanings, batched over cells:

  Context.OB_step(Iapp)              <- OB_step.m:1        (cellState lives in the context)
  Context.iterEKF(vk, ik)            <- iterEKF.m:30       (ekfData lives in the context)
  Context.EKFmatsHandler(zk, Xind)   <- EKFmatsHandler.m:1
  Context.iterMPC(lin, SOCk_1)       <- iterMPC.m:1        (mpcData lives in the context)
  predMat(a, C, D, Np, Nc)           <- predMat.m:1        (A = diag(a), B = ones)
  constraintsMPC(lin, uk_1, SOCk_1)  <- constraintsMPC.m:1
  hildreth(E, F, M, gamma, lambda0, maxIter) <- hildreth.m:1
  runMPC(rom, SOC0, TC, nsteps)      <- runMPC.m:72-112    (fused, batched)

Errors: MATLAB ``error()`` becomes :class:`MpcekfError`; per-cell soft failures
(EKF lock-out, thetae < 0) set ``status`` bits and make that cell's outputs NaN.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import LIN_SIZE, MpcekfError, check, dptr, iptr
from .rom import EL_TABLES, ROM, TF_CODE

__all__ = ["Context", "DeviceBuffer", "hip_runtimes", "tc_grid", "make_config", "predMat", "constraintsMPC", "hildreth", "runMPC", "MpcekfError",
           "LIN_SIZE"]

LIN_FIELDS = dict(A=slice(0, 6), Csoc=slice(6, 12), Dsoc=12, Cv=slice(13, 19), Dv=19,
                  Cphi=slice(20, 26), Dphi=26, bv=27, bphi=28, xhat=slice(29, 35))


def make_config(**kw) -> _lib.Config:
    """mpcekf_config with the runMPC.m defaults, overridden by keyword."""
    L = _lib.load()
    c = _lib.Config()
    L.mpcekf_config_defaults(C.byref(c))
    alias = {"targetSOC": "target_soc", "maxHild": "max_hild"}
    for k, v in kw.items():
        k = alias.get(k, k)
        if k == "constraints":
            c.use_current, c.use_voltage, c.use_eta = (int(x) for x in v)
        elif k == "SigmaX0":
            for i in range(6):
                c.SigmaX0[i] = float(v[i])
        elif k == "method":
            # initKF.m:44-49 blend selector: 'OB'/'OutB' (runMPC.m:16) or 'MB'/'MdlB'
            m = str(v).upper()
            if m not in ("OB", "OUTB", "MB", "MDLB"):
                raise ValueError(f"method {v!r}: expected 'OB' or 'MB' (initKF.m:44-49)")
            c.method = _lib.METHOD_MB if m in ("MB", "MDLB") else _lib.METHOD_OB
        elif k == "bounds":
            c.flags = (c.flags | _lib.CF_BOUNDS) if v else (c.flags & ~_lib.CF_BOUNDS)
        else:
            if not hasattr(c, k):
                raise TypeError(f"unknown config field {k}")
            setattr(c, k, type(getattr(c, k))(v))
    return c


class _PackedRom:
    def __init__(self, rom: ROM):
        self.keep = []

        def arr(x, dt=np.float64):
            a = np.ascontiguousarray(x, dtype=dt)
            self.keep.append(a)
            return a

        r = _lib.Rom()
        r.nT, r.nZ, r.n, r.nz = rom.nT, rom.nZ, rom.n, rom.nz
        r.T_degC = dptr(arr(rom.T_degC))
        r.SOC_pct = dptr(arr(rom.SOC_pct))
        r.Ts = rom.Ts
        r.A = dptr(arr(rom.A))
        r.C = dptr(arr(rom.C))
        r.D = dptr(arr(rom.D))
        r.tf_code = iptr(arr([TF_CODE[n] for n in rom.names], np.int32))
        r.tf_xloc = dptr(arr(rom.xloc))
        r.F, r.R, r.Q, r.Rc, r.Tref = rom.F, rom.R, rom.Q, rom.Rc, rom.Tref
        r.tab_ntheta, r.tab_ntemp = rom.ntheta, rom.ntemp
        r.tab_T_K = dptr(arr(np.atleast_1d(rom.tab_T_K)))
        for side in ("neg", "pos"):
            e = getattr(rom, side)
            s = getattr(r, side)
            s.theta0, s.theta100 = e.theta0, e.theta100
            for k in ("soc0", "soc100", "Uocp", "dUocp", "k0", "Rf", "Cdleff", "Uocp1"):
                setattr(s, k, dptr(arr(getattr(e, k))))
            for k in EL_TABLES + ("Uocp1",):    # ABI v3 theta polynomials (NULL: v2 linear tables)
                has = bool(e.poly) and k in e.poly
                setattr(s, k + "_p", dptr(arr(e.poly[k])) if has else _lib._dp())
            for i, k in enumerate(EL_TABLES):  # ABI v3 Arrhenius energies (0: none)
                s.Ea[i] = float((e.Ea or {}).get(k, 0.0))
            for i, k in enumerate(EL_TABLES + ("Uocp1",)):  # ABI v4: functions on their own nodes
                if e.nodes and k in e.nodes:
                    x, c = e.nodes[k]
                    c = np.asarray(c, dtype=np.float64)
                    if c.shape[-1] < rom.npoly:   # one coefficient count (tab_npoly): zero-padded
                        c = np.concatenate([c, np.zeros(c.shape[:-1] + (rom.npoly - c.shape[-1],))], -1)
                    s.nnode[i] = int(np.asarray(x).size)
                    s.node[i] = dptr(arr(x))
                    s.node_p[i] = dptr(arr(c))
        r.tab_npoly = rom.npoly
        self.s = r


def tc_grid(tc, nsteps, ncells):
    """A temperature argument as the [nsteps, ncells] grid of per-step TC (degC): a scalar,
    a 1-D per-step profile [nsteps] or per-cell vector [ncells], [nsteps, 1], [1, ncells]
    or the full array.  A 1-D vector whose length is both nsteps and ncells is ambiguous
    and refused (oracle/oracle_c.py reads temperature arguments by the same rule)."""
    a = np.asarray(tc, dtype=np.float64)
    if a.ndim == 1 and a.size != 1:
        if a.size == nsteps and a.size == ncells:
            raise ValueError(f"tc: a 1-D vector of length {a.size} = nsteps = ncells is ambiguous; "
                             "pass [nsteps, 1] (per step) or [1, ncells] (per cell)")
        if a.size == nsteps:
            a = a.reshape(nsteps, 1)
        elif a.size == ncells:
            a = a.reshape(1, ncells)
        else:
            raise ValueError(f"tc: length {a.size} is neither nsteps ({nsteps}) nor ncells ({ncells})")
    return np.ascontiguousarray(np.broadcast_to(a, (nsteps, ncells)))


class DeviceBuffer:
    """A C-contiguous device array allocated by the library's own HIP runtime
    (mpcekf_dev_alloc), for outputs_on_device calls: the host process then holds one
    HIP runtime only, and no foreign runtime's pointers reach the kernels."""

    def __init__(self, shape, dtype=np.float64, device=0):
        self.L = _lib.load()
        self.shape = tuple(int(x) for x in np.atleast_1d(shape))
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = C.c_void_p()
        check(self.L.mpcekf_dev_alloc(int(device), self.nbytes, C.byref(p)))
        self.ptr = p.value or 0

    def free(self):
        if getattr(self, "ptr", 0):
            self.L.mpcekf_dev_free(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.free()

    def row_bytes(self):
        return self.nbytes // self.shape[0] if self.shape and self.shape[0] else 0

    def to_host(self, rows=None):
        """The first ``rows`` leading-axis rows (default all) as a numpy array."""
        rows = self.shape[0] if rows is None else int(rows)
        if not 0 <= rows <= self.shape[0]:
            raise ValueError(f"to_host: rows = {rows} outside [0, {self.shape[0]}]")
        out = np.empty((rows,) + self.shape[1:], dtype=self.dtype)
        check(self.L.mpcekf_dev_copy(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr), out.nbytes,
                                     _lib.COPY_D2H))
        return out

    def sampled(self, rows, stride):
        """[rows, ncells] buffer -> its every ``stride``-th column of the first ``rows`` rows
        (a pitched device-to-host copy: only the sampled elements cross PCIe)."""
        if len(self.shape) != 2 or stride < 1 or self.shape[1] % stride:
            raise ValueError("sampled: 2-D buffer with ncells divisible by stride expected")
        n = self.shape[1]
        rows = int(rows)
        if not 0 <= rows <= self.shape[0]:
            raise ValueError(f"sampled: rows = {rows} outside [0, {self.shape[0]}]")
        it = self.dtype.itemsize
        out = np.empty((rows, n // stride), dtype=self.dtype)
        check(self.L.mpcekf_dev_copy2d(out.ctypes.data_as(C.c_void_p), it, C.c_void_p(self.ptr), stride * it, it,
                                       rows * (n // stride), _lib.COPY_D2H))
        return out

    def from_host(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        if a.nbytes > self.nbytes:
            raise ValueError("from_host: array larger than the buffer")
        check(self.L.mpcekf_dev_copy(C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p), a.nbytes, _lib.COPY_H2D))


def hip_runtimes():
    """Paths of the HIP / HSA runtime libraries mapped into this process ({'hip': [...],
    'hsa': [...]}): one of each when the library's runtime is the only one."""
    out = {"hip": set(), "hsa": set()}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.split() else ""
                if "libamdhip64" in p:
                    out["hip"].add(p)
                elif "libhsa-runtime64" in p:
                    out["hsa"].add(p)
    except OSError:
        pass
    return {k: sorted(v) for k, v in out.items()}


class Context:
    """One device, one stream, ``ncells`` independent cells (mpcekf_ctx)."""

    def __init__(self, rom: ROM, ncells: int, cfg: _lib.Config | None = None, device: int = 0):
        self.L = _lib.load()
        self.rom = rom
        self.cfg = cfg if cfg is not None else make_config()
        self.device = device
        self._pr = _PackedRom(rom)
        h = C.c_void_p()
        check(self.L.mpcekf_ctx_create(C.byref(self._pr.s), C.byref(self.cfg), device, int(ncells), C.byref(h)))
        self.h = h
        n, nm, nz, nc = C.c_int64(), C.c_int32(), C.c_int32(), C.c_int32()
        check(self.L.mpcekf_ctx_info(h, C.byref(n), C.byref(nm), C.byref(nz), C.byref(nc)))
        self.n, self.NM, self.nz, self.ncon = n.value, nm.value, nz.value, nc.value
        # asynchronous = True: the stage functions below call the _async C-ABI twins (SURVEY.md
        # §8(b)): they return before their host outputs are written; sync() (or any synchronous
        # stage call) completes them.  The output arrays are held here until then.
        self.asynchronous = False
        self._pending = []

    def _stage(self, name, *args, keep=()):
        """One stage entry point: mpcekf_<name>, or mpcekf_<name>_async in asynchronous mode
        (its output arrays `keep` held until the synchronisation)."""
        if self.asynchronous:
            check(getattr(self.L, f"mpcekf_{name}_async")(self.h, *args))
            self._pending.append(keep)
        else:
            check(getattr(self.L, f"mpcekf_{name}")(self.h, *args))
            self._pending.clear()

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.L.mpcekf_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _vec(self, x, dtype=np.float64):
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(x, dtype=dtype), (self.n,)))
        return a

    # -- initKF / initMPC / first OB_step --------------------------------
    def init_cells(self, soc0_pct, tc_degC):
        s = self._vec(soc0_pct)
        t = self._vec(tc_degC)
        check(self.L.mpcekf_init_cells(self.h, dptr(s), dptr(t)))

    # -- fused loop (runMPC.m:83-112) ------------------------------------
    # runMPC.m stores per step: name -> (dtype, trailing shape); see mpcekf_traj
    TRAJ_FIELDS = dict(u=(np.float64, ()), v=(np.float64, ()), soc=(np.float64, ()), phise=(np.float64, ()),
                       nexec=(np.int32, ()), x=(np.float64, (6,)), zk=(np.float64, None),
                       zbk=(np.float64, None), J_unc=(np.float64, ()), J_fin=(np.float64, ()),
                       norm_du=(np.float64, ()), nviol=(np.int32, ()), poles=(np.float64, (7, 2)),
                       sv=(np.float64, (7,)))

    def step(self, nsteps, outputs=("u", "v", "soc", "phise", "nexec"), tc=None):
        """nsteps fused closed-loop steps (runMPC.m:83-112).  ``outputs`` names the per-step
        stores to return as [nsteps, ncells(, k)] arrays: u, v, soc, phise, nexec, and the
        diagnostics x (x_store), zk / zbk (zkEst / zkBound), J_unc, J_fin, norm_du, nviol
        (mpcData.cost), poles ([.., 7, 2] re/im of eig(CL)) and sv (svd(CL)), the stability
        diagnostics of iterMPC.m:53-60 (returned as complex [nsteps, ncells, 7] for poles).
        ``tc``: the TC of each step in degC (runMPC.m:85-92), see :func:`tc_grid`; None keeps
        every cell's current temperature."""
        n = self.n
        tcs = None if tc is None else tc_grid(tc, nsteps, n)
        out = {}
        tr = _lib.Traj()
        for k in outputs:
            if k not in self.TRAJ_FIELDS:
                raise KeyError(f"unknown output {k}")
            dt, tail = self.TRAJ_FIELDS[k]
            tail = (self.nz + 2,) if tail is None else tail
            out[k] = np.empty((nsteps, n) + tail, dtype=dt)
            setattr(tr, k, out[k].ctypes.data_as(C.c_void_p).value)
        check(self.L.mpcekf_step_ex(self.h, int(nsteps), tcs.ctypes.data_as(C.c_void_p) if tcs is not None else None,
                                    C.byref(tr), 0))
        if "poles" in out:
            out["poles"] = _complex(out["poles"])
        return out

    def step_device(self, nsteps, u=0, v=0, soc=0, phise=0, nexec=0):
        """Fused steps writing [nsteps][ncells] outputs to device pointers (ints or
        DeviceBuffer; allocate them with DeviceBuffer / mpcekf_dev_alloc)."""
        p = [C.c_void_p(x.ptr if isinstance(x, DeviceBuffer) else x) if x else None for x in (u, v, soc, phise, nexec)]
        check(self.L.mpcekf_step(self.h, int(nsteps), None, *p, 1))

    def sync(self):
        """Wait for every launch on the context's device and complete the asynchronous stage
        calls' host outputs (mpcekf_sync)."""
        check(self.L.mpcekf_sync(self.h))
        self._pending.clear()

    def set_graph(self, enable=True):
        """Replay repeated fused-call shapes from captured hipGraphs (mpcekf_set_graph)."""
        check(self.L.mpcekf_set_graph(self.h, int(bool(enable))))

    def set_timing(self, enable=True):
        """enable: True/1 = every step; N > 1 = sample every N-th step (less perturbation)."""
        check(self.L.mpcekf_set_timing(self.h, int(enable)))

    def get_timing(self):
        """{kernel: (ms_sum, launches)} since the last call (HIP events on the ctx stream)."""
        names = ("plant", "flush", "cell", "hild", "bounds")  # MPCEKF_K_* order
        ms = np.zeros(len(names))
        nl = (C.c_int64 * len(names))()
        check(self.L.mpcekf_get_timing(self.h, dptr(ms), nl))
        return {k: (float(ms[i]), int(nl[i])) for i, k in enumerate(names)}

    def get_stamps(self):
        """k_cell section stamps of the last fused step [NSTAMPS][ncells] (profiling builds; else None)."""
        ns = C.c_int32(0)
        check(self.L.mpcekf_get_stamps(self.h, None, C.byref(ns)))
        if ns.value == 0:
            return None
        out = np.empty((ns.value, self.n), dtype=np.int64)
        check(self.L.mpcekf_get_stamps(self.h, out.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(ns)))
        return out

    def get_hild_problems(self):
        """(prob [51][ncells] field-major, hflag [ncells]) of the last fused step (diagnostic)."""
        prob = np.empty((51, self.n))
        hflag = np.empty(self.n, dtype=np.int32)
        check(self.L.mpcekf_get_hild_problems(self.h, dptr(prob), iptr(hflag)))
        return prob, hflag

    def get_zk(self):
        zk = np.empty((self.n, self.nz + 2))
        zb = np.empty((self.n, self.nz + 2))
        check(self.L.mpcekf_get_zk(self.h, dptr(zk), dptr(zb)))
        return zk, zb

    # -- MATLAB-named stage functions --------------------------------------
    def _tvec(self, T):
        return None if T is None else self._vec(T)

    def OB_step(self, Iapp, Tc=None):
        """[Vcell, ~, cellState] = OB_step(Iapp, Tc, cellState, ROM)  (OB_step.m:1).
        Tc (degC, scalar or [n]) becomes the cell temperature; None keeps the current one."""
        i = self._vec(Iapp)
        t = self._tvec(Tc)
        v = np.empty(self.n)
        self._stage("plant_step", dptr(i), dptr(t), dptr(v), keep=(v,))
        return v

    def iterEKF(self, vk, ik, Tk=None, bounds=True, xind=True):
        """[zk, boundzk, ekfData, Xind] = iterEKF(vk, ik, Tk, ekfData)  (iterEKF.m:30).

        Xind is returned as dict(model=[n,4] model index t*nZ+z, theT, theZ, gamma);
        xind=False: None (it stays on the device for EKFmatsHandler(None, None)).  vk = None:
        the last OB_step's Vcell on the device (the asynchronous route's hand-off)."""
        v = None if vk is None else self._vec(vk)
        i = self._vec(ik)
        t = self._tvec(Tk)
        zk = np.empty((self.n, self.nz + 2))
        zb = np.empty((self.n, self.nz + 2)) if bounds else None
        xm = np.empty((self.n, 4), dtype=np.int32) if xind else None
        xg = np.empty((self.n, 4)) if xind else None
        self._stage("ekf_step", dptr(v), dptr(i), dptr(t), dptr(zk), dptr(zb), iptr(xm), dptr(xg), keep=(zk, zb, xm, xg))
        if not xind:
            return zk, zb, None
        return zk, zb, _Xind(model=xm, gamma=xg, nZ=self.rom.nZ)

    def EKFmatsHandler(self, zk, Xind, Tk=None, keep=False):
        """[MPC, xhat] = EKFmatsHandler(ekfData, Xind, zk, Tk)  (EKFmatsHandler.m:1).

        Returns the packed linearisation records [n, 35] (fields: LIN_FIELDS).  zk = Xind =
        None: the device copies of the last iterEKF; keep=True: the records stay on the
        device only (None is returned; lin_fields reads slots, iterMPC / mpc_diag take
        lin=None) -- the stage route without host round trips."""
        t = self._tvec(Tk)
        lin = None if keep else np.empty((self.n, LIN_SIZE))
        if zk is None:
            self._stage("linearize", None, None, None, dptr(t), dptr(lin), keep=(lin,))
            return lin
        zk = np.ascontiguousarray(zk, dtype=np.float64)
        xm = np.ascontiguousarray(Xind["model"], dtype=np.int32)
        xg = np.ascontiguousarray(Xind["gamma"], dtype=np.float64)
        self._stage("linearize", dptr(zk), iptr(xm), dptr(xg), dptr(t), dptr(lin), keep=(lin,))
        return lin

    def lin_fields(self, slots, set=None, out=None):
        """Slots (MPCEKF_LIN_*) of the device-resident records of the last EKFmatsHandler:
        [n, len(slots)]; ``set`` [n, len(slots)] is written into them first.  ``out``: a
        C-contiguous float64 [n, len(slots)] array to fill instead of a new one."""
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        if out is None:
            out = np.empty((self.n, sl.size))
        elif out.shape != (self.n, sl.size) or out.dtype != np.float64 or not out.flags.c_contiguous:
            raise ValueError(f"lin_fields: out must be a C-contiguous float64 array of shape {(self.n, sl.size)}")
        st = None
        if set is not None:
            st = np.ascontiguousarray(set, dtype=np.float64)
            if st.size != self.n * sl.size:   # the C side reads n * len(slots) doubles from it
                raise ValueError(f"lin_fields: set must hold {(self.n, sl.size)} values, got shape {st.shape}")
            st = st.reshape(self.n, sl.size)
        self._stage("lin_fields", iptr(sl), int(sl.size), dptr(st), dptr(out), keep=(out,))
        return out

    def iterMPC(self, lin, SOCk_1, cost=False):
        """[uk, mpcData] = iterMPC(xk, cellState, mpcData)  (iterMPC.m:1). Returns uk, nexec;
        with cost=True also this call's mpcData.cost row (iterMPC.m:89-95) as a dict of
        J_uncon, J_final, norm_DU, viol, nexec per cell."""
        lin = None if lin is None else np.ascontiguousarray(lin, dtype=np.float64)   # None: the device record
        s = None if SOCk_1 is None else self._vec(SOCk_1)   # None: zk(end) of the last iterEKF, on the device
        uk = np.empty(self.n)
        ne = np.empty(self.n, dtype=np.int32)
        if not cost:
            self._stage("mpc_step", dptr(lin), dptr(s), dptr(uk), iptr(ne), keep=(uk, ne))
            return uk, ne
        ju, jf, nd = np.empty(self.n), np.empty(self.n), np.empty(self.n)
        nv = np.empty(self.n, dtype=np.int32)
        self._stage("mpc_step_ex", dptr(lin), dptr(s), dptr(uk), iptr(ne), dptr(ju), dptr(jf), dptr(nd), iptr(nv),
                    keep=(uk, ne, ju, jf, nd, nv))
        return uk, ne, dict(J_uncon=ju, J_final=jf, norm_DU=nd, viol=nv, nexec=ne)

    def mpc_diag(self, lin, uk_1=None):
        """mpcData.poles / mpcData.sv of the iterMPC that iterMPC(lin, ..) would run
        (iterMPC.m:53-60): (poles complex [n, 7], sv [n, 7]).  uk_1 None: the context's."""
        lin = None if lin is None else np.ascontiguousarray(lin, dtype=np.float64)   # None: the device record
        u = None if uk_1 is None else self._vec(uk_1)
        p = np.empty((self.n, 7, 2))
        sv = np.empty((self.n, 7))
        self._stage("mpc_diag", dptr(lin), dptr(u), dptr(p), dptr(sv), keep=(p, sv))
        return _complex(p), sv   # a view of p: asynchronously, its values arrive at the sync

    # -- state -----------------------------------------------------------
    def get_state(self):
        n, NM = self.n, self.NM
        st = dict(bigX=np.empty((n, NM, 6)), ekf=np.empty((n, NM, 20)), scal=np.empty((n, _lib.NSCAL)),
                  lam=np.empty((n, self.ncon)), warn=np.empty(n, np.int32), status=np.empty(n, np.int32))
        if self.cfg.method == _lib.METHOD_MB:
            st["mb"] = np.empty((n, _lib.MB_SIZE))
        s = _lib.State(dptr(st["bigX"]), dptr(st["ekf"]), dptr(st["scal"]), dptr(st["lam"]),
                       iptr(st["warn"]), iptr(st["status"]), dptr(st.get("mb")))
        check(self.L.mpcekf_get_state(self.h, C.byref(s)))
        return st

    SCALARS = ("SOCnAvg", "SOCpAvg", "x0", "SigmaX0", "priorI", "uk_1", "uk", "vk")  # MPCEKF_S_* order

    def get_scalars(self, names=("SOCnAvg", "SOCpAvg"), flags=False):
        """The named per-cell scalars ({name: [ncells]}; names from SCALARS) and, with
        flags=True, warn / status -- only these bytes cross PCIe (mpcekf_get_scalars)."""
        slots = np.array([self.SCALARS.index(k) for k in names], dtype=np.int32)
        sc = np.empty((self.n, len(slots)))
        warn = np.empty(self.n, np.int32) if flags else None
        status = np.empty(self.n, np.int32) if flags else None
        self._stage("get_scalars", iptr(slots), len(slots), dptr(sc), iptr(warn), iptr(status), keep=(sc, warn, status))
        out = {k: sc[:, j] for j, k in enumerate(names)}
        if flags:
            out.update(warn=warn, status=status)
        return out

    def set_state(self, st):
        a = {k: (np.ascontiguousarray(v, dtype=np.int32 if k in ("warn", "status") else np.float64)
                 if v is not None else None) for k, v in st.items()}
        s = _lib.State(dptr(a.get("bigX")), dptr(a.get("ekf")), dptr(a.get("scal")), dptr(a.get("lam")),
                       iptr(a.get("warn")), iptr(a.get("status")), dptr(a.get("mb")))
        check(self.L.mpcekf_set_state(self.h, C.byref(s)))


def _complex(p):
    """[..., 2] re / im float64 pairs as a complex128 [...] view (no copy, the exact pairs:
    re + 1j * im would turn a -0 real part into +0 and an infinite imaginary part's real
    part into NaN)."""
    return p.view(np.complex128)[..., 0]


class _Xind(dict):
    """iterEKF's Xind: model / gamma, and theT / theZ (model // nZ, model % nZ) formed when
    first read -- after an asynchronous iterEKF, model holds its values only after the sync."""

    def __init__(self, model, gamma, nZ):
        super().__init__(model=model, gamma=gamma)
        self._nZ = nZ

    def __missing__(self, key):
        if key == "theT":
            v = self["model"] // self._nZ
        elif key == "theZ":
            v = self["model"] % self._nZ
        else:
            raise KeyError(key)
        self[key] = v
        return v


# ---------------------------------------------------------------------------
# context-free batched functions
# ---------------------------------------------------------------------------
def predMat(a, Cr, D, Np=5, Nc=2, device=0):
    """predMat.m with A = diag(a) (a [n,6]), B = ones, C [n,6], D [n] -> Phi [n,Np,7], G [n,Np,Nc]."""
    L = _lib.load()
    a = np.ascontiguousarray(np.atleast_2d(a), dtype=np.float64)
    Cr = np.ascontiguousarray(np.atleast_2d(Cr), dtype=np.float64)
    D = np.ascontiguousarray(np.atleast_1d(D), dtype=np.float64)
    n = a.shape[0]
    Phi = np.empty((n, Np, 7))
    G = np.empty((n, Np, Nc))
    check(L.mpcekf_predmat(device, n, Np, Nc, dptr(a), dptr(Cr), dptr(D), dptr(Phi), dptr(G)))
    return Phi, G


def constraintsMPC(lin, uk_1, SOCk_1, Q, cfg=None, device=0):
    """constraintsMPC.m: lin [n,35] -> M [n,ncon,Nc], gamma [n,ncon]."""
    L = _lib.load()
    cfg = cfg if cfg is not None else make_config()
    lin = np.ascontiguousarray(np.atleast_2d(lin), dtype=np.float64)
    n = lin.shape[0]
    u = np.ascontiguousarray(np.broadcast_to(uk_1, (n,)), dtype=np.float64)
    s = np.ascontiguousarray(np.broadcast_to(SOCk_1, (n,)), dtype=np.float64)
    ncon = 4 * cfg.Nc + 3 * cfg.Np
    M = np.empty((n, ncon, cfg.Nc))
    g = np.empty((n, ncon))
    check(L.mpcekf_constraints(device, C.byref(cfg), float(Q), n, dptr(lin), dptr(u), dptr(s), dptr(M), dptr(g)))
    return M, g


def hildreth(E, F, M, gamma, lambda0=None, maxIter=100, tol=1e-6, device=0):
    """hildreth.m batched: E [n,Nc,Nc], F [n,Nc], M [n,ncon,Nc], gamma [n,ncon]."""
    L = _lib.load()
    E = np.ascontiguousarray(E, dtype=np.float64)
    n, Nc = E.shape[0], E.shape[1]
    F = np.ascontiguousarray(F, dtype=np.float64)
    M = np.ascontiguousarray(M, dtype=np.float64)
    g = np.ascontiguousarray(gamma, dtype=np.float64)
    ncon = M.shape[1]
    lam = np.zeros((n, ncon)) if lambda0 is None else np.array(lambda0, dtype=np.float64, order="C")
    DU = np.empty((n, Nc))
    ne = np.empty(n, dtype=np.int32)
    check(L.mpcekf_hildreth(device, n, Nc, ncon, dptr(E), dptr(F), dptr(M), dptr(g), dptr(lam),
                            int(maxIter), float(tol), dptr(DU), iptr(ne)))
    return DU, lam, ne


def hildreth_structured(E, F, Hv, He, Hs, gamma, lambda0=None, maxIter=100, tol=1e-6, device=0):
    """hildreth.m on constraintsMPC.m-structured problems (the fused step's solver):
    E [n,2,2], F [n,2], Hv/He/Hs [n,5] Toeplitz columns, gamma [n,23]."""
    L = _lib.load()
    E = np.ascontiguousarray(E, dtype=np.float64)
    n = E.shape[0]
    a = [np.ascontiguousarray(x, dtype=np.float64) for x in (F, Hv, He, Hs, gamma)]
    lam = np.zeros((n, 23)) if lambda0 is None else np.array(lambda0, dtype=np.float64, order="C")
    DU = np.empty((n, 2))
    ne = np.empty(n, dtype=np.int32)
    check(L.mpcekf_hildreth_structured(device, n, dptr(E), *[dptr(x) for x in a], dptr(lam), int(maxIter),
                                       float(tol), dptr(DU), iptr(ne)))
    return DU, lam, ne


def structured_M(Hv, He, Hs):
    """The constraintsMPC.m matrix [Cu; -Cu; I; -I; G_v; -G_e; G_soc] (23 x 2) of
    Toeplitz columns, with the kernels' exact entries (signed zeros included)."""
    M = np.zeros((23, 2))
    for i in range(2):
        for k in range(2):
            M[i, k] = 1.0 if k <= i else 0.0
            M[2 + i, k] = -(1.0 if k <= i else 0.0)
            M[4 + i, k] = 1.0 if i == k else 0.0
            M[6 + i, k] = -(1.0 if i == k else 0.0)
    for r in range(5):
        for k in range(2):
            M[8 + r, k] = Hv[r - k] if k <= r else 0.0
            M[13 + r, k] = -(He[r - k] if k <= r else 0.0)
            M[18 + r, k] = Hs[r - k] if k <= r else 0.0
    return M


def runMPC(rom, SOC0, TC, nsteps, cfg=None, device=0, ncells=None, tc_traj=None):
    """runMPC.m:72-112 for a batch of cells; returns trajectories [nsteps, ncells].
    tc_traj [nsteps, ncells] (degC): a temperature profile (TC is the initial one)."""
    SOC0 = np.atleast_1d(np.asarray(SOC0, dtype=np.float64))
    n = ncells or SOC0.shape[0]
    with Context(rom, n, cfg, device) as ctx:
        ctx.init_cells(SOC0, TC)
        out = ctx.step(nsteps, tc=tc_traj)
        out["status"] = ctx.get_state()["status"]
        return out


def cl_eig(a):
    """eig / svd of one small square matrix as the fused step computes mpcData.poles and
    mpcData.sv (iterMPC.m:57-60; mpcekf_cl_eig): (poles complex [n] sorted by descending
    real then imaginary part, sv [n] descending).  Host code, no device needed."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    n = a.shape[0]
    if a.shape != (n, n):
        raise ValueError("square matrix expected")
    re, im, sv = np.empty(n), np.empty(n), np.empty(n)
    L = _lib.load()
    check(L.mpcekf_cl_eig(n, dptr(a), dptr(re), dptr(im), dptr(sv)))
    return re + 1j * im, sv
