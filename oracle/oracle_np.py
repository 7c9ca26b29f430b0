"""oracle/oracle_np.py -- CPU restatement of the reference hot path in numpy.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``mpc-ekf4fastcharge_amd/``)
imports, links or executes this file; only ``tests/``, ``tools/make_golden.py``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it,
and only as the checker.

PARITY UNPINNED: the reference is MATLAB (no MATLAB/Octave in this image) and
ships no tests, fixtures or golden vectors; its ROM file ROM_NMC30_HRA.mat is
missing (.MISSING_LARGE_BLOBS:1).  This restatement therefore runs on the
synthetic ROM of ``rom.py`` and is pinned only by analytic known-answer tests
(tests/test_oracle.py, the KATs of its first half) and by agreement with the independent C
restatement (oracle/mpcekf_oracle.c).  See DESIGN.md "Oracle".

Conventions (identical in the C oracle and the kernels):
* every dot product / matrix product is a sequential sum starting from +0.0
  over the inner index in ascending order (reference BLAS ddot order), with
  no fused multiply-add;
* MATLAB ``max/min`` ignore NaN (fmax/fmin semantics);
* ``E\\b`` with E symmetric with positive diagonal -> Cholesky (MATLAB
  mldivide), ``-E\\b`` parses as ``(-E)\\b`` -> LU with partial pivoting;
* this file keeps the full 5x5 covariances and uses LAPACK ``svd`` for the
  symmetrisation step (iterEKF.m:143-145), i.e. it is the MATLAB-faithful
  variant; the C oracle keeps packed covariances and a Jacobi eigensolver.

Functions mirror the reference one-to-one and cite it by file:line.
"""
from __future__ import annotations

import math

import numpy as np

NAN = float("nan")

# status bits (include/mpcekf.h MPCEKF_ST_*)
ST_ERROR = 1
ST_LOCKOUT = 2
ST_THETAE_NEG = 4


# ---------------------------------------------------------------------------
# defined-order linear algebra helpers
# ---------------------------------------------------------------------------
def mv(A, x):
    """y = A*x, y_i = ((0 + A_i1 x_1) + A_i2 x_2) + ...  (vectorised over i)."""
    A = np.asarray(A, dtype=float)
    acc = np.zeros(A.shape[0])
    for k in range(A.shape[1]):
        acc = acc + A[:, k] * x[k]
    return acc


def mm(A, B):
    """C = A*B with sequential inner sums from 0."""
    A = np.asarray(A, dtype=float)
    B = np.asarray(B, dtype=float)
    acc = np.zeros((A.shape[0], B.shape[1]))
    for k in range(A.shape[1]):
        acc = acc + A[:, k:k + 1] * B[k:k + 1, :]
    return acc


def _sqrt(x):
    return math.sqrt(x) if x >= 0 else NAN


def dot(a, b):
    acc = 0.0
    for x, y in zip(a, b):
        acc = acc + x * y
    return acc


def chol_solve(E, B):
    """E\\B via Cholesky (upper R, E = R'R) -- MATLAB mldivide for SPD E.

    Returns None when the factorisation fails (non-positive pivot)."""
    n = E.shape[0]
    R = np.zeros((n, n))
    for j in range(n):
        s = E[j, j]
        for k in range(j):
            s = s - R[k, j] * R[k, j]
        if not (s > 0):
            return None
        R[j, j] = math.sqrt(s)
        for i in range(j + 1, n):
            t = E[j, i]
            for k in range(j):
                t = t - R[k, j] * R[k, i]
            R[j, i] = t / R[j, j]
    B = np.array(B, dtype=float)
    vec = B.ndim == 1
    if vec:
        B = B[:, None]
    X = np.zeros_like(B)
    for c in range(B.shape[1]):
        y = np.zeros(n)
        for i in range(n):
            t = B[i, c]
            for k in range(i):
                t = t - R[k, i] * y[k]
            y[i] = t / R[i, i]
        for i in range(n - 1, -1, -1):
            t = y[i]
            for k in range(i + 1, n):
                t = t - R[i, k] * X[k, c]
            X[i, c] = t / R[i, i]
    return X[:, 0] if vec else X


def lu_solve(A, b):
    """A\\b via LU with partial pivoting (first max on ties), dgesv-like."""
    A = np.array(A, dtype=float)
    y = np.array(b, dtype=float)
    n = A.shape[0]
    for k in range(n):
        p = k
        for i in range(k + 1, n):
            if abs(A[i, k]) > abs(A[p, k]):
                p = i
        if p != k:
            A[[k, p], :] = A[[p, k], :]
            y[[k, p]] = y[[p, k]]
        for i in range(k + 1, n):
            l = A[i, k] / A[k, k]
            A[i, k] = l
            for j in range(k + 1, n):
                A[i, j] = A[i, j] - l * A[k, j]
    for i in range(n):
        for k in range(i):
            y[i] = y[i] - A[i, k] * y[k]
    x = np.zeros(n)
    for i in range(n - 1, -1, -1):
        t = y[i]
        for k in range(i + 1, n):
            t = t - A[i, k] * x[k]
        x[i] = t / A[i, i]
    return x


def mldivide_spd(E, B):
    """MATLAB ``E\\B`` for symmetric E with positive diagonal: chol, else LU."""
    X = chol_solve(E, B)
    if X is None:
        B = np.asarray(B, dtype=float)
        if B.ndim == 1:
            return lu_solve(E, B)
        return np.stack([lu_solve(E, B[:, c]) for c in range(B.shape[1])], axis=1)
    return X


def stable_two_nearest(d):
    """[~,i] = sort(d) (stable, NaN last); return i(1), i(2)."""
    order = np.argsort(np.asarray(d, dtype=float), kind="stable")
    return int(order[0]), int(order[1]) if len(order) > 1 else int(order[0])


# ---------------------------------------------------------------------------
# cellData.function.* (tabulated semantics, see rom.py)
# ---------------------------------------------------------------------------
class Cell:
    """Reads the ROM *data*; re-implements the tabulated handle semantics itself
    (include/mpcekf.h mpcekf_electrode): [ntemp, ntheta] tables, theta interpolated
    on a uniform [0, 1] grid (linearly, or by the v3 piecewise polynomials) or, for a
    function with ABI v4 nodes, by its polynomials on its own theta nodes; then T linearly
    between the two bracketing grid rows, then the v3 Arrhenius factor.

    ``handles=True``: calls the ROM's closed-form ``cellData.function`` handles
    (``rom.handles``, rom.py SynthHandles) instead, at every call site, as MATLAB does --
    the reference semantics the tables approximate."""

    def __init__(self, rom, handles=False):
        self.rom = rom
        self.F = rom.F
        self.R = rom.R
        self.Q = rom.Q
        self.Rc = rom.Rc
        self.Tref = rom.Tref
        self.TK = [float(t) for t in np.atleast_1d(rom.tab_T_K)]
        self.e = {"neg": rom.neg, "pos": rom.pos}
        self.h = None
        if handles:
            self.h = getattr(rom, "handles", None)
            if self.h is None:
                raise ValueError("handle mode needs a ROM with closed-form handles (rom.handles)")

    @staticmethod
    def _interp(tab, x):
        if x != x:
            return NAN
        n = len(tab)
        xc = min(max(x, 0.0), 1.0)
        t = xc * (n - 1)
        i = int(math.floor(t))
        if i > n - 2:
            i = n - 2
        f = t - i
        return float(tab[i] + f * (tab[i + 1] - tab[i]))

    @staticmethod
    def _poly(coef, x):
        """v3 row: Horner c0 + s (c1 + s (... + s c_last)) on interval i of the uniform grid."""
        if x != x:
            return NAN
        n = len(coef) + 1
        xc = min(max(x, 0.0), 1.0)
        t = xc * (n - 1)
        i = int(math.floor(t))
        if i > n - 2:
            i = n - 2
        s = t - i
        c = coef[i]
        v = float(c[-1])                     # Horner: c0 + s (c1 + s (... + s c_last))
        for k in range(len(c) - 2, -1, -1):
            v = float(c[k] + s * v)
        return v

    @staticmethod
    def _node(x, coef, th):
        """ABI v4 row (include/mpcekf.h mpcekf_electrode.nnode): the polynomial of segment k on
        the function's own nodes x [m], k the last of 0..m-2 with k = 0 or x_k <= theta
        (theta clamped to [0, 1]; a linear scan here, the C oracle bisects), s = theta - x_k."""
        if th != th:
            return NAN
        xc = min(max(th, 0.0), 1.0)
        k = 0
        while k + 1 <= len(x) - 2 and x[k + 1] <= xc:
            k += 1
        s = xc - float(x[k])
        c = coef[k]
        v = float(c[-1])
        for q in range(len(c) - 2, -1, -1):
            v = float(c[q] + s * v)
        return v

    def _fn(self, s, name, th, T):
        """One v3 lookup: rows (polynomial or linear) bilinear in T, times the Arrhenius factor.
        A function with v4 nodes uses its own node polynomials for the rows instead."""
        e = self.e[s]
        nd = e.nodes.get(name) if getattr(e, "nodes", None) else None
        coef = nd[1] if nd is not None else (e.poly.get(name) if e.poly else None)
        tab = getattr(e, name)
        j, g = self._tj(T)
        if nd is not None:
            row = lambda k: self._node(nd[0], coef[k], th)
        else:
            row = (lambda k: self._interp(tab[k], th)) if coef is None else (lambda k: self._poly(coef[k], th))
        one = coef is not None and all(np.array_equal(coef[0], coef[k]) for k in range(1, len(coef)))
        v = row(0 if one else j)               # T-invariant rows: row 0, no blend
        if len(self.TK) > 1 and not one:
            b = row(j + 1)
            v = v + g * (b - v)
        ea = float(e.Ea.get(name, 0.0)) if e.Ea else 0.0
        if ea != 0.0:
            v = v * _dexp((ea / self.R) * (1.0 / self.Tref - 1.0 / T))
        return v

    def _tj(self, T):
        TK = self.TK
        if len(TK) == 1:
            return 0, 0.0
        Tc = min(max(T, TK[0]), TK[-1])
        j = 0
        while j < len(TK) - 2 and Tc >= TK[j + 1]:
            j += 1
        return j, (Tc - TK[j]) / (TK[j + 1] - TK[j])

    def soc(self, s, z, T):
        if self.h is not None:
            return self.h[s].soc(z, T)
        e = self.e[s]
        j, g = self._tj(T)
        if len(self.TK) == 1:
            s0, s1 = float(e.soc0[0]), float(e.soc100[0])
        else:
            s0 = e.soc0[j] + g * (e.soc0[j + 1] - e.soc0[j])
            s1 = e.soc100[j] + g * (e.soc100[j + 1] - e.soc100[j])
        return s0 + z * (s1 - s0)

    def Uocp(self, s, th, T=None):
        if self.h is not None:
            return self.h[s].Uocp(th, T)
        if T is None:                                  # one-argument call (EKFmatsHandler.m:96)
            e = self.e[s]
            if getattr(e, "nodes", None) and "Uocp1" in e.nodes:
                return self._node(*e.nodes["Uocp1"], th)
            return self._poly(e.poly["Uocp1"], th) if e.poly else self._interp(e.Uocp1, th)
        return self._fn(s, "Uocp", th, T)

    def dUocp(self, s, th, T):
        return self.h[s].dUocp(th, T) if self.h is not None else self._fn(s, "dUocp", th, T)

    def k0(self, s, th, T):
        return self.h[s].k0(th, T) if self.h is not None else self._fn(s, "k0", th, T)

    def Rf(self, s, th, T):
        return self.h[s].Rf(th, T) if self.h is not None else self._fn(s, "Rf", th, T)

    def Cdleff(self, s, th, T):
        """Cdl(th,T)^(2-nDL) * wDL(th,T)^(nDL-1) (OB_step.m:212-219), tabulated by the exporter."""
        return self.h[s].Cdleff(th, T) if self.h is not None else self._fn(s, "Cdleff", th, T)


# the defined exp of the v3 Arrhenius factor (rom.py dexp; kernels dexp; C oracle orc_exp)
_EXP_P = (1.66666666666666019037e-01, -2.77777777770155933842e-03, 6.61375632143793436117e-05,
          -1.65339022054652515390e-06, 4.13813679705723846039e-08)


def _dexp(x):
    if x != x:
        return x
    if x > 709.782712893384:
        return math.inf
    if x < -745.1332191019412:
        return 0.0
    k = math.floor(x * 1.44269504088896338700e+00 + 0.5)
    hi = x - k * 6.93147180369123816490e-01
    lo = k * 1.90821492927058770002e-10
    r = hi - lo
    t = r * r
    P1, P2, P3, P4, P5 = _EXP_P
    c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))))
    y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi)
    return math.ldexp(y, int(k))


# ---------------------------------------------------------------------------
# index setup (iterEKF.m:610-735; OB_step.m:86-163)
# ---------------------------------------------------------------------------
def setup_inds(rom):
    names = list(rom.names)
    loc = np.asarray(rom.xloc, dtype=float)

    def f(nm):
        return [i for i, s in enumerate(names) if s == nm]

    ind = {nm: f(nm) for nm in set(names)}
    for nm in ("negIfdl", "posIfdl", "negIf", "posIf", "negIdl", "posIdl", "negPhis", "posPhis",
               "negPhise", "posPhise", "negThetass", "posThetass", "negPhie", "sepPhie", "posPhie",
               "negThetae", "sepThetae", "posThetae"):
        ind.setdefault(nm, [])
    ind["Ifdl"] = ind["negIfdl"] + ind["posIfdl"]
    ind["If"] = ind["negIf"] + ind["posIf"]
    ind["Phise"] = ind["negPhise"] + ind["posPhise"]
    ind["Thetass"] = ind["negThetass"] + ind["posThetass"]
    ind["Phie"] = ind["negPhie"] + ind["sepPhie"] + ind["posPhie"]
    ind["Thetae"] = ind["negThetae"] + ind["sepThetae"] + ind["posThetae"]
    pick = lambda lst, x: [i for i in lst if loc[i] == x][0]
    ind["Ifdl0"], ind["Ifdl3"] = pick(ind["Ifdl"], 0), pick(ind["Ifdl"], 3)
    ind["If0"], ind["If3"] = pick(ind["If"], 0), pick(ind["If"], 3)
    ind["Thetass0"], ind["Thetass3"] = pick(ind["Thetass"], 0), pick(ind["Thetass"], 3)
    ind["Phise0"] = pick(ind["Phise"], 0)
    locPhie = [loc[i] for i in ind["Phie"]]
    if locPhie[0] == 0:                                        # iterEKF.m:728-731
        ind["Phie"] = ind["Phie"][1:]
        locPhie = locPhie[1:]
    ind["locPhie"] = locPhie
    return ind


# ---------------------------------------------------------------------------
# OB_step (plant), OB_step.m:1-357
# ---------------------------------------------------------------------------
def ob_step_init(rom, SOC0_pct, Tc, handles=False):
    """First call of OB_step (OB_step.m:39-72): returns cellState."""
    cell = Cell(rom, handles)
    ind = setup_inds(rom)
    NM = rom.NM
    bigA = np.zeros((rom.n + 1, NM))
    Cfull = np.zeros((NM, rom.nz, rom.n + 1))
    Dfull = np.zeros((NM, rom.nz))
    for tt in range(rom.nT):
        for zz in range(rom.nZ):
            col = tt * rom.nZ + zz
            bigA[:, col] = rom.A[tt, zz]
            C = rom.C[tt, zz].copy()
            C[ind["negPhise"], -1] = 0.0                        # OB_step.m:178
            if ind["posPhise"]:
                C[ind["posPhise"], -1] = 0.0                    # OB_step.m:179-181
            Cfull[col] = C
            Dfull[col] = rom.D[tt, zz]
    Tk1 = Tc + 273.15
    SOC0n = cell.soc("neg", SOC0_pct / 100, Tk1)
    SOC0p = cell.soc("pos", SOC0_pct / 100, Tk1)
    return dict(cell=cell, ind=ind, bigA=bigA, bigX=np.zeros_like(bigA), C=Cfull, D=Dfull,
                Tspts=np.sort(rom.T_degC) + 273.15, Zspts=np.sort(rom.SOC_pct / 100), ZZ=rom.nZ,
                Ts=rom.Ts, SOCnAvg=SOC0n, SOCpAvg=SOC0p, SOC0n=SOC0n, SOC0p=SOC0p)


def ob_step(Iapp, Tc, cs):
    """One simStep (OB_step.m:188-357). Mutates cs; returns Vcell."""
    cell = cs["cell"]
    ind = cs["ind"]
    T = Tc + 273.15                                            # OB_step.m:75
    F, R, Q, Rc = cell.F, cell.R, cell.Q, cell.Rc
    e_n, e_p = cell.e["neg"], cell.e["pos"]
    theta0n, theta0p, theta100n, theta100p = e_n.theta0, e_p.theta0, e_n.theta100, e_p.theta100
    Cdleffn = cell.Cdleff("neg", cs["SOC0n"], T)               # OB_step.m:212-219 at SOC0n/p
    Cdleffp = cell.Cdleff("pos", cs["SOC0p"], T)
    SOCnAvg, SOCpAvg = cs["SOCnAvg"], cs["SOCpAvg"]
    negSOC, posSOC = SOCnAvg, SOCpAvg
    cellSOC = (SOCnAvg - theta0n) / (theta100n - theta0n)      # OB_step.m:228
    dUocpnAvg = cell.dUocp("neg", SOCnAvg, T)
    dUocppAvg = cell.dUocp("pos", SOCpAvg, T)
    dQn = abs(theta100n - theta0n)
    dQp = abs(theta100p - theta0p)
    res0n = -dQn / (3600 * Q - Cdleffn * dQn * dUocpnAvg)      # OB_step.m:235
    res0p = dQp / (3600 * Q - Cdleffp * dQp * dUocppAvg)
    Ts = cs["Ts"]
    SOCnAvg = SOCnAvg + res0n * Iapp * Ts                      # OB_step.m:239-244
    SOCpAvg = SOCpAvg + res0p * Iapp * Ts
    if SOCnAvg < 0:
        SOCnAvg = 0.0
    if SOCnAvg > 1:
        SOCnAvg = 1.0
    if SOCpAvg < 0:
        SOCpAvg = 0.0
    if SOCpAvg > 1:
        SOCpAvg = 1.0
    Zspts, Tspts, ZZ = cs["Zspts"], cs["Tspts"], cs["ZZ"]
    if len(Zspts) > 1:                                          # OB_step.m:251-259
        a, b = stable_two_nearest(np.abs(cellSOC - Zspts))
        iZu, iZl = max(a, b), min(a, b)
    else:
        iZu = iZl = 0
    Zu, Zl = Zspts[iZu], Zspts[iZl]
    if len(Tspts) > 1:
        a, b = stable_two_nearest(np.abs(T - Tspts))
        iTu, iTl = max(a, b), min(a, b)
    else:
        iTu = iTl = 0
    Tu, Tl = Tspts[iTu], Tspts[iTl]
    bigX = cs["bigX"]
    Cm, Dm = cs["C"], cs["D"]

    def yk_of(it, iz):
        col = it * ZZ + iz
        return mv(Cm[col], bigX[:, col]) + Dm[col] * Iapp      # OB_step.m:272-275

    yk1, yk2, yk3, yk4 = yk_of(iTl, iZl), yk_of(iTl, iZu), yk_of(iTu, iZl), yk_of(iTu, iZu)
    cs["bigX"] = cs["bigA"] * bigX + Iapp                       # OB_step.m:278
    aZ = 0.0
    aT = 0.0
    if Zu != Zl:
        aZ = (cellSOC - Zl) / (Zu - Zl)
    if Tu != Tl:
        aT = (T - Tl) / (Tu - Tl)
    yk = (1 - aT) * ((1 - aZ) * yk1 + aZ * yk2) + aT * ((1 - aZ) * yk3 + aZ * yk4)
    negIfdl0 = yk[ind["Ifdl0"]]
    posIfdl3 = yk[ind["Ifdl3"]]
    negIf0 = yk[ind["If0"]]
    posIf3 = yk[ind["If3"]]
    clamp = lambda x: min(max(x, 1e-6), 1 - 1e-6) if x == x else min(1e-6, 1 - 1e-6)
    negThetass0 = clamp(yk[ind["Thetass0"]] + cs["SOC0n"])     # OB_step.m:304-310
    posThetass3 = clamp(yk[ind["Thetass3"]] + cs["SOC0p"])
    th1 = yk[ind["Thetae"][0]] + 1
    thE = yk[ind["Thetae"][-1]] + 1
    Thetae1 = th1 if th1 >= 1e-6 else 1e-6                      # max(x,1e-6), NaN -> 1e-6
    ThetaeE = thE if thE >= 1e-6 else 1e-6
    k0n = cell.k0("neg", negSOC, T)
    k0p = cell.k0("pos", posSOC, T)
    i0n = k0n * _sqrt(Thetae1 * (1 - negThetass0) * negThetass0)
    i0p = k0p * _sqrt(ThetaeE * (1 - posThetass3) * posThetass3)
    negEta0 = 2 * R * T / F * math.asinh(negIf0 / (2 * i0n))
    posEta3 = 2 * R * T / F * math.asinh(posIf3 / (2 * i0p))
    Uocpn0 = cell.Uocp("neg", negThetass0, T)
    Uocpp3 = cell.Uocp("pos", posThetass3, T)
    Rfn = cell.Rf("neg", negSOC, T)
    Rfp = cell.Rf("pos", posSOC, T)
    Vcell = (posEta3 - negEta0 + yk[ind["Phie"][-1]] + Uocpp3 - Uocpn0
             + (Rfp * posIfdl3 - Rfn * negIfdl0))               # OB_step.m:341-342
    Vcell = Vcell - Rc * Iapp
    cs["SOCnAvg"], cs["SOCpAvg"] = SOCnAvg, SOCpAvg
    return Vcell


# ---------------------------------------------------------------------------
# initKF (initKF.m:30-136) and iterEKF 'OB' (iterEKF.m:30-210)
# ---------------------------------------------------------------------------
def init_kf(rom, SOC0, T0, SigmaX0, SigmaV, SigmaW, method="OB", handles=False):
    """initKF.m:30-136.  method 'OB' (output blend) or 'MB' (model blend, initKF.m:44-49)."""
    n = rom.n
    method = {"OUTB": "OB", "OB": "OB", "MDLB": "MB", "MB": "MB"}[method.upper()]
    if SigmaX0.shape != (n + 1, n + 1):
        raise ValueError("SigmaX0 has wrong dimension (initKF.m:66-69)")
    if T0 > 100:
        T0 = T0 - 273.15
    TK = rom.mdl_T_K()
    ZS = rom.mdl_Z()
    M = {}
    for t in range(rom.nT):
        for z in range(rom.nZ):
            M[(t, z)] = dict(A=rom.A[t, z, :n].copy(), C=rom.C[t, z, :, :n].copy(),
                             D=rom.D[t, z].copy(), xhat=np.zeros(n),
                             SigmaX=np.array(SigmaX0[:n, :n], dtype=float))
    return dict(rom=rom, cell=Cell(rom, handles), ind=setup_inds(rom), M=M, n=n, nz=rom.nz,
                x0=0.0, SigmaX0=float(SigmaX0[n, n]), xhat=np.zeros(n + 1),
                SigmaV=SigmaV, SigmaW=SigmaW, priorI=0.0, Ts=rom.Ts, SOC0=SOC0 / 100,
                Q=rom.Q, Tpts=np.unique(TK), Zpts=np.unique(ZS), warnCount=0, status=0,
                method=method, SigmaX=np.array(SigmaX0, dtype=float))   # initKF.m:100-101 (MB)


def get_xind(ekf, Tk, SOC):
    """iterEKF.m:219-255."""
    Zpts, Tpts = ekf["Zpts"], ekf["Tpts"]
    if len(Zpts) > 1:
        i1, i2 = stable_two_nearest(np.abs(SOC - Zpts))
        iZu, iZl = i1, i2
        if Zpts[iZu] < Zpts[iZl]:
            iZu, iZl = i2, i1
    else:
        iZu = iZl = 0
    if len(Tpts) > 1:
        i1, i2 = stable_two_nearest(np.abs(Tk - Tpts))
        iTu, iTl = i1, i2
        if Tpts[iTu] < Tpts[iTl]:
            iTu, iTl = i2, i1
    else:
        iTu = iTl = 0
    aZ = 0.0
    aT = 0.0
    if len(Zpts) > 1:
        aZ = (SOC - Zpts[iZl]) / (Zpts[iZu] - Zpts[iZl])
    if len(Tpts) > 1:
        aT = (Tk - Tpts[iTl]) / (Tpts[iTu] - Tpts[iTl])
    gamma = [(1 - aT) * (1 - aZ), (1 - aT) * aZ, aT * (1 - aZ), aT * aZ]
    return dict(gamma=gamma, theT=[iTl, iTl, iTu, iTu], theZ=[iZl, iZu, iZl, iZu])


def _warn(ekf):
    ekf["warnCount"] += 1                                       # iterEKF.m:741-751


def get_variables(ekf, ik, Xind, T):
    """iterEKF.m:259-417 ('OB').  Returns (Vcell, Z, Zsoc)."""
    cell, ind = ekf["cell"], ekf["ind"]
    F, R = cell.F, cell.R
    mdl = [ekf["M"][(Xind["theT"][j], Xind["theZ"][j])] for j in range(4)]
    mb = ekf["method"] == "MB"
    x0 = ekf["xhat"][-1] if mb else ekf["x0"]                   # iterEKF.m:265-275
    xSOC = ekf["SOC0"] - x0 * (ekf["Ts"] / (3600 * ekf["Q"]))
    SOCnAvg = cell.soc("neg", xSOC, T)
    SOCpAvg = cell.soc("pos", xSOC, T)
    if SOCnAvg < 0:
        _warn(ekf)
        SOCnAvg = 1e-6
    if SOCnAvg > 1:
        _warn(ekf)
        SOCnAvg = 1 - 1e-6
    if SOCpAvg < 0:
        _warn(ekf)
        SOCpAvg = 1e-6
    if SOCpAvg > 0.998:
        _warn(ekf)
        SOCpAvg = 0.998
    Z = np.zeros(ekf["nz"])
    for j in range(4):                                          # iterEKF.m:312-313
        xj = ekf["xhat"][:-1] if mb else mdl[j]["xhat"]         # MB: iterEKF.m:314-315
        zj = mv(mdl[j]["C"], xj) + mdl[j]["D"] * ik
        Z = Z + zj * Xind["gamma"][j]
    If0 = Z[ind["If0"]]
    If3 = Z[ind["If3"]]
    nt, pt = ind["negThetass"], ind["posThetass"]
    Z[nt] = Z[nt] + SOCnAvg
    if np.any(Z[nt] < 0):
        _warn(ekf)
        v = Z[nt]
        v[v < 0] = 1e-6
        Z[nt] = v
    if np.any(Z[nt] > 1):
        _warn(ekf)
        v = Z[nt]
        v[v > 1] = 1 - 1e-6
        Z[nt] = v
    Z[pt] = Z[pt] + SOCpAvg
    if np.any(Z[pt] < 0):
        _warn(ekf)
        v = Z[pt]
        v[v < 0] = 1e-6
        Z[pt] = v
    if np.any(Z[pt] > 0.998):
        _warn(ekf)
        v = Z[pt]
        v[v > 0.998] = 0.998
        Z[pt] = v
    UocpnAvg = cell.Uocp("neg", SOCnAvg, T)
    UocppAvg = cell.Uocp("pos", SOCpAvg, T)
    Z[ind["negPhise"]] = Z[ind["negPhise"]] + UocpnAvg
    if ind["posPhise"]:
        Z[ind["posPhise"]] = Z[ind["posPhise"]] + UocppAvg
    PhieTilde3 = Z[ind["Phie"][-1]]
    Phise0 = Z[ind["Phise0"]]
    for k, r in enumerate(ind["Phie"]):                         # iterEKF.m:373-379
        if ind["locPhie"][k] == 0:
            Z[r] = 0 - Phise0
        else:
            Z[r] = Z[r] - Phise0
    Z[ind["Thetae"]] = Z[ind["Thetae"]] + 1
    if np.any(Z[ind["Thetae"]] < 0):                            # iterEKF.m:384-389: MATLAB errors
        _warn(ekf)
        ekf["status"] |= ST_ERROR | ST_THETAE_NEG
        return NAN, np.full(ekf["nz"], NAN), NAN
    k0n = cell.k0("neg", SOCnAvg, T)
    k0p = cell.k0("pos", SOCpAvg, T)
    i0n = k0n * _sqrt(Z[ind["Thetae"][0]] * (1 - Z[ind["Thetass0"]]) * Z[ind["Thetass0"]])
    i0p = k0p * _sqrt(Z[ind["Thetae"][-1]] * (1 - Z[ind["Thetass3"]]) * Z[ind["Thetass3"]])
    negEta0 = 2 * R * T / F * math.asinh(If0 / (2 * i0n))
    posEta3 = 2 * R * T / F * math.asinh(If3 / (2 * i0p))
    Uocpn0 = cell.Uocp("neg", Z[ind["Thetass0"]], T)
    Uocpp3 = cell.Uocp("pos", Z[ind["Thetass3"]], T)
    Rfn = cell.Rf("neg", SOCnAvg, T)
    Rfp = cell.Rf("pos", SOCpAvg, T)
    Vcell = (posEta3 - negEta0 + PhieTilde3 + Uocpp3 - Uocpn0
             + (Rfp * Z[ind["Ifdl3"]] - Rfn * Z[ind["Ifdl0"]]))  # iterEKF.m:409-410
    Z[ind["posPhis"]] = Z[ind["posPhis"]] + Vcell
    Zsoc = ekf["SOC0"] - x0 * (ekf["Ts"] / (3600 * ekf["Q"]))
    return Vcell, Z, Zsoc


def get_chat_v(ekf, Xind, Z, Tk):
    """iterEKF.m:421-519 ('OB'). Returns (Chat[4] of length n, Chat0)."""
    cell, ind = ekf["cell"], ekf["ind"]
    F, R = cell.F, cell.R
    Cs = [Xind["gamma"][j] * ekf["M"][(Xind["theT"][j], Xind["theZ"][j])]["C"] for j in range(4)]
    if ekf["method"] == "MB":
        return _get_chat_v_mb(ekf, Cs, Z, Tk)
    x0 = ekf["x0"]
    xSOC = ekf["SOC0"] - x0 * (ekf["Ts"] / (3600 * ekf["Q"]))
    SOCnAvg = cell.soc("neg", xSOC, Tk)
    SOCpAvg = cell.soc("pos", xSOC, Tk)
    Rfn = cell.Rf("neg", SOCnAvg, Tk)
    Rfp = cell.Rf("pos", SOCpAvg, Tk)
    Chat = [Rfp * C[ind["Ifdl3"]] - Rfn * C[ind["Ifdl0"]] for C in Cs]
    k0n = cell.k0("neg", SOCnAvg, Tk)
    k0p = cell.k0("pos", SOCpAvg, Tk)
    i0n = k0n * _sqrt(Z[ind["Thetae"][0]] * (1 - Z[ind["Thetass0"]]) * Z[ind["Thetass0"]])
    i0p = k0p * _sqrt(Z[ind["Thetae"][-1]] * (1 - Z[ind["Thetass3"]]) * Z[ind["Thetass3"]])
    Rctn = R * Tk / (F * i0n)
    Rctp = R * Tk / (F * i0p)
    Chat = [Chat[j] + Rctp * Cs[j][ind["If3"]] - Rctn * Cs[j][ind["If0"]] for j in range(4)]
    Chat = [Chat[j] + Cs[j][ind["Phie"][-1]] for j in range(4)]
    dUocpn0 = cell.dUocp("neg", Z[ind["Thetass0"]], Tk)
    dUocpp3 = cell.dUocp("pos", Z[ind["Thetass3"]], Tk)
    Ts, Q = ekf["Ts"], ekf["Q"]
    res0n = -dUocpn0 * Ts * (cell.soc("neg", 1, Tk) - cell.soc("neg", 0, Tk)) / (3600 * Q)
    res0p = -dUocpp3 * Ts * (cell.soc("pos", 1, Tk) - cell.soc("pos", 0, Tk)) / (3600 * Q)
    Chat0 = res0p - res0n
    Chat = [Chat[j] + (dUocpp3 * Cs[j][ind["Thetass3"]] - dUocpn0 * Cs[j][ind["Thetass0"]])
            for j in range(4)]
    return Chat, Chat0


def _sum4(rows):
    """MATLAB sum([r1; r2; r3; r4]) down the columns, in row order."""
    return ((rows[0] + rows[1]) + rows[2]) + rows[3]


def _get_chat_v_mb(ekf, Cs, Z, Tk):
    """getChatV 'MB' branches (iterEKF.m:448-459, 475-479, 489-491, 512-517): one blended
    voltage row over the shared state, augmented with the integrator term -> (Chat[n+1], Chat0)."""
    cell, ind = ekf["cell"], ekf["ind"]
    F, R = cell.F, cell.R
    Ts, Q = ekf["Ts"], ekf["Q"]
    x0 = ekf["xhat"][-1]
    xSOC = ekf["SOC0"] - x0 * (Ts / (3600 * Q))
    SOCnAvg = cell.soc("neg", xSOC, Tk)
    SOCpAvg = cell.soc("pos", xSOC, Tk)
    Rfn = cell.Rf("neg", SOCnAvg, Tk)
    Rfp = cell.Rf("pos", SOCpAvg, Tk)
    rows = lambda r: _sum4([C[r] for C in Cs])
    Chat = Rfp * rows(ind["Ifdl3"]) - Rfn * rows(ind["Ifdl0"])
    k0n = cell.k0("neg", SOCnAvg, Tk)
    k0p = cell.k0("pos", SOCpAvg, Tk)
    i0n = k0n * _sqrt(Z[ind["Thetae"][0]] * (1 - Z[ind["Thetass0"]]) * Z[ind["Thetass0"]])
    i0p = k0p * _sqrt(Z[ind["Thetae"][-1]] * (1 - Z[ind["Thetass3"]]) * Z[ind["Thetass3"]])
    Rctn = R * Tk / (F * i0n)
    Rctp = R * Tk / (F * i0p)
    Chat = Chat + Rctp * rows(ind["If3"]) - Rctn * rows(ind["If0"])
    Chat = Chat + rows(ind["Phie"][-1])
    dUocpn0 = cell.dUocp("neg", Z[ind["Thetass0"]], Tk)
    dUocpp3 = cell.dUocp("pos", Z[ind["Thetass3"]], Tk)
    res0n = -dUocpn0 * Ts * (cell.soc("neg", 1, Tk) - cell.soc("neg", 0, Tk)) / (3600 * Q)
    res0p = -dUocpp3 * Ts * (cell.soc("pos", 1, Tk) - cell.soc("pos", 0, Tk)) / (3600 * Q)
    Chat0 = res0p - res0n
    Chat = Chat + dUocpp3 * rows(ind["Thetass3"]) - dUocpn0 * rows(ind["Thetass0"])
    return np.concatenate([Chat, [Chat0]]), Chat0


def get_chat_z(ekf, Xind, Z, Tk):
    """iterEKF.m:523-602 ('OB'; 'MB' in _get_chat_z_mb)."""
    cell, ind = ekf["cell"], ekf["ind"]
    Cs = [Xind["gamma"][j] * ekf["M"][(Xind["theT"][j], Xind["theZ"][j])]["C"] for j in range(4)]
    if ekf["method"] == "MB":
        return _get_chat_z_mb(ekf, Xind, Cs, Z, Tk)
    Chat = [C.copy() for C in Cs]
    Chat0 = np.zeros(ekf["nz"])
    ChatV, ChatV0 = get_chat_v(ekf, Xind, Z, Tk)
    for kk in range(4):
        C = Chat[kk]
        for r in ind["posPhis"]:
            C[r] = C[r] + ChatV[kk]
        Chat[kk] = C
    Chat0[ind["posPhis"]] = ChatV0
    Ts, Q = ekf["Ts"], ekf["Q"]
    res0n = -Ts * (cell.soc("neg", 1, Tk) - cell.soc("neg", 0, Tk)) / (3600 * Q)
    res0p = -Ts * (cell.soc("pos", 1, Tk) - cell.soc("pos", 0, Tk)) / (3600 * Q)
    Chat0[ind["negThetass"]] = res0n
    Chat0[ind["posThetass"]] = res0p
    x0 = ekf["x0"]
    xSOC = ekf["SOC0"] - x0 * (Ts / (3600 * Q))
    SOCnAvg = cell.soc("neg", xSOC, Tk)
    SOCpAvg = cell.soc("pos", xSOC, Tk)
    dUocpn = cell.dUocp("neg", SOCnAvg, Tk)
    dUocpp = cell.dUocp("pos", SOCpAvg, Tk)
    Chat0[ind["negPhise"]] = dUocpn * res0n
    Chat0[ind["posPhise"]] = dUocpp * res0p
    Chat0[ind["Phie"]] = -dUocpn * res0n
    for kk in range(4):
        C = Chat[kk]
        for r in ind["Phie"]:
            C[r] = C[r] - C[ind["Phise0"]]
        Chat[kk] = C
    return Chat, ChatV, Chat0, ChatV0


def _get_chat_z_mb(ekf, Xind, Cs, Z, Tk):
    """getChatZ 'MB' branches (iterEKF.m:537-538, 554-558, 575-576, 596-600) -> (Chat nz x (n+1),
    ChatV n+1, Chat0 nz, ChatV0)."""
    cell, ind = ekf["cell"], ekf["ind"]
    Chat = ((Cs[0] + Cs[1]) + Cs[2]) + Cs[3]
    Chat0 = np.zeros(ekf["nz"])
    ChatV, ChatV0 = get_chat_v(ekf, Xind, Z, Tk)
    for r in ind["posPhis"]:
        Chat[r] = Chat[r] + ChatV[:-1]
    Chat0[ind["posPhis"]] = ChatV[-1]
    Ts, Q = ekf["Ts"], ekf["Q"]
    res0n = -Ts * (cell.soc("neg", 1, Tk) - cell.soc("neg", 0, Tk)) / (3600 * Q)
    res0p = -Ts * (cell.soc("pos", 1, Tk) - cell.soc("pos", 0, Tk)) / (3600 * Q)
    Chat0[ind["negThetass"]] = res0n
    Chat0[ind["posThetass"]] = res0p
    xSOC = ekf["SOC0"] - ekf["xhat"][-1] * (Ts / (3600 * Q))
    dUocpn = cell.dUocp("neg", cell.soc("neg", xSOC, Tk), Tk)
    dUocpp = cell.dUocp("pos", cell.soc("pos", xSOC, Tk), Tk)
    Chat0[ind["negPhise"]] = dUocpn * res0n
    Chat0[ind["posPhise"]] = dUocpp * res0p
    Chat0[ind["Phie"]] = -dUocpn * res0n
    for r in ind["Phie"]:
        Chat[r] = Chat[r] - Chat[ind["Phise0"]]
    return np.concatenate([Chat, Chat0[:, None]], axis=1), ChatV, Chat0, ChatV0


def _symmetrise_bump(S, residual, St):
    """iterEKF.m:142-154 / 164-173: svd symmetrisation, then the Q-bump."""
    _, SS, VVh = np.linalg.svd(S)
    VV = VVh.T
    HH = (VV * SS[None, :]) @ VV.T
    S = (S + S.T + HH + HH.T) / 4
    if residual ** 2 > 9 * St:
        S = S * 2
    return S


def _iter_ekf_mb(ekf, vk, ik, Tk):
    """iterEKF.m:30-210 with method 'MB': one blended model over one (n+1) state and one
    (n+1)x(n+1) covariance per cell (iterEKF.m:90-102, 125-128, 160-176, 199-203)."""
    nz, n = ekf["nz"], ekf["n"]
    r = ekf["Ts"] / (3600 * ekf["Q"])
    W = ekf["SigmaW"]
    SOC = ekf["SOC0"] - ekf["xhat"][-1] * r                     # iterEKF.m:92-93
    Xind = get_xind(ekf, Tk, SOC)
    As = [ekf["M"][(Xind["theT"][j], Xind["theZ"][j])]["A"] for j in range(4)]
    g = Xind["gamma"]
    AMB = np.concatenate([((As[0] * g[0] + As[1] * g[1]) + As[2] * g[2]) + As[3] * g[3], [1.0]])
    ekf["xhat"] = AMB * ekf["xhat"] + ekf["priorI"]
    ekf["SigmaX"] = (AMB[:, None] * ekf["SigmaX"]) * AMB[None, :] + W
    SOC = ekf["SOC0"] - ekf["xhat"][-1] * r
    Xind = get_xind(ekf, Tk, SOC)
    vhat, Z, _ = get_variables(ekf, ik, Xind, Tk)
    if ekf["status"] & ST_ERROR:
        return np.full(nz + 2, NAN), np.full(nz + 2, NAN), None
    ChatV, _ = get_chat_v(ekf, Xind, Z, Tk)                     # iterEKF.m:125-128
    S = ekf["SigmaX"]
    St = dot(mv(S.T, ChatV), ChatV) + ekf["SigmaV"]
    L = mv(S, ChatV) / St
    residual = vk - vhat
    ekf["xhat"] = ekf["xhat"] + L * residual                     # iterEKF.m:160-173
    LS = L * St
    ekf["SigmaX"] = _symmetrise_bump(S - LS[:, None] * L[None, :], residual, St)
    SOC = ekf["SOC0"] - ekf["xhat"][-1] * r
    Xind = get_xind(ekf, Tk, SOC)
    vhat, Z, Zsoc = get_variables(ekf, ik, Xind, Tk)
    if ekf["status"] & ST_ERROR:
        return np.full(nz + 2, NAN), np.full(nz + 2, NAN), None
    zk = np.concatenate([Z, [vhat, Zsoc]])
    res = -r
    ChatZ, ChatVz, _, _ = get_chat_z(ekf, Xind, zk, Tk)         # iterEKF.m:199-203 (diag only)
    S = ekf["SigmaX"]
    P = mm(ChatZ, S)
    SigZ = np.zeros(nz)
    for c in range(n + 1):
        SigZ = SigZ + P[:, c] * ChatZ[:, c]
    SigV = dot(mv(S.T, ChatVz), ChatVz)
    SigSOC = res * S[-1, -1] * res
    with np.errstate(invalid="ignore"):
        boundzk = 3 * np.sqrt(np.concatenate([SigZ, [SigV, SigSOC]]))
    ekf["priorI"] = ik
    return zk, boundzk, Xind


def iter_ekf(ekf, vk, ik, Tk):
    """iterEKF.m:30-210 with method 'OB' ('MB' in _iter_ekf_mb). Returns (zk, boundzk, Xind)."""
    nz = ekf["nz"]
    if ekf["status"] & ST_ERROR:
        return np.full(nz + 2, NAN), np.full(nz + 2, NAN), None
    if ekf["warnCount"] > 10:                                   # iterEKF.m:55-59
        ekf["status"] |= ST_LOCKOUT | ST_ERROR
        return np.full(nz + 2, NAN), np.full(nz + 2, NAN), None
    if Tk > 100:
        pass
    else:
        Tk = Tk + 273.15
    if ekf["method"] == "MB":
        return _iter_ekf_mb(ekf, vk, ik, Tk)
    W = ekf["SigmaW"]
    for key, m in ekf["M"].items():                             # iterEKF.m:73-84
        A = m["A"]
        m["xhat"] = A * m["xhat"] + ekf["priorI"]
        m["SigmaX"] = (A[:, None] * m["SigmaX"]) * A[None, :] + W
    ekf["x0"] = ekf["x0"] + ekf["priorI"]
    ekf["SigmaX0"] = ekf["SigmaX0"] + W
    SOC = ekf["SOC0"] - ekf["x0"] * (ekf["Ts"] / (3600 * ekf["Q"]))
    Xind = get_xind(ekf, Tk, SOC)
    vhat, Z, _ = get_variables(ekf, ik, Xind, Tk)
    if ekf["status"] & ST_ERROR:
        return np.full(nz + 2, NAN), np.full(nz + 2, NAN), None
    ChatV, C0 = get_chat_v(ekf, Xind, Z, Tk)                    # iterEKF.m:114-124
    S1 = ekf["M"][(Xind["theT"][0], Xind["theZ"][0])]["SigmaX"]
    SV = ekf["SigmaV"]
    St, L = [], []
    for j in range(4):
        row = mv(S1.T, ChatV[j])          # ChatV*SigmaX (1x5): t_c = sum_r c_r S_rc
        s = dot(row, ChatV[j]) + SV
        St.append(s)
        L.append(mv(S1, ChatV[j]) / s)
    SigmaX0 = ekf["SigmaX0"]
    St0 = C0 * SigmaX0 * C0 + SV
    L0 = SigmaX0 * C0 / St0
    residual = vk - vhat
    for j in range(4):                                          # iterEKF.m:136-154
        m = ekf["M"][(Xind["theT"][j], Xind["theZ"][j])]
        m["xhat"] = m["xhat"] + L[j] * residual
        LS = L[j] * St[j]
        S = m["SigmaX"] - LS[:, None] * L[j][None, :]
        _, SS, VVh = np.linalg.svd(S)
        VV = VVh.T
        HH = (VV * SS[None, :]) @ VV.T
        S = (S + S.T + HH + HH.T) / 4
        if residual ** 2 > 9 * St[j]:
            S = S * 2
        m["SigmaX"] = S
    ekf["x0"] = ekf["x0"] + L0 * residual
    ekf["SigmaX0"] = ekf["SigmaX0"] - L0 * St0 * L0
    SOC = ekf["SOC0"] - ekf["x0"] * (ekf["Ts"] / (3600 * ekf["Q"]))
    Xind = get_xind(ekf, Tk, SOC)
    vhat, Z, Zsoc = get_variables(ekf, ik, Xind, Tk)
    if ekf["status"] & ST_ERROR:
        return np.full(nz + 2, NAN), np.full(nz + 2, NAN), None
    zk = np.concatenate([Z, [vhat, Zsoc]])
    res = -ekf["Ts"] / (3600 * ekf["Q"])
    ChatZ, ChatVz, ChatZ0, ChatV0 = get_chat_z(ekf, Xind, zk, Tk)
    S1 = ekf["M"][(Xind["theT"][0], Xind["theZ"][0])]["SigmaX"]
    SigZ = np.zeros(nz)
    SigV = 0.0
    for j in range(4):                                          # iterEKF.m:191-195 (diag only)
        P = mm(ChatZ[j], S1)
        q = np.zeros(nz)
        for c in range(ekf["n"]):
            q = q + P[:, c] * ChatZ[j][:, c]
        SigZ = SigZ + q
        SigV = SigV + dot(mv(S1.T, ChatVz[j]), ChatVz[j])
    SigZ = SigZ + (ChatZ0 * ekf["SigmaX0"]) * ChatZ0
    SigV = SigV + ChatV0 * ekf["SigmaX0"] * ChatV0
    SigSOC = res * ekf["SigmaX0"] * res
    with np.errstate(invalid="ignore"):
        boundzk = 3 * np.sqrt(np.concatenate([SigZ, [SigV, SigSOC]]))
    ekf["priorI"] = ik
    return zk, boundzk, Xind


# ---------------------------------------------------------------------------
# EKFmatsHandler (EKFmatsHandler.m:1-115)
# ---------------------------------------------------------------------------
def ekf_mats_handler(ekf, Xind, zk, Tk):
    cell, ind = ekf["cell"], ekf["ind"]
    g = Xind["gamma"]
    imax = 0
    for j in range(1, 4):                                       # max(): first on ties, NaN ignored
        if g[j] > g[imax] or (g[imax] != g[imax] and g[j] == g[j]):
            imax = j
    mdl = ekf["M"][(Xind["theT"][imax], Xind["theZ"][imax])]
    xhat = np.concatenate([mdl["xhat"], [ekf["xhat"][-1]]])
    a = np.concatenate([mdl["A"], [1.0]])
    nx = len(a)
    C, D = mdl["C"], mdl["D"]
    r = -ekf["Ts"] / (3600 * ekf["Q"])
    Csoc = np.zeros(nx)
    Csoc[-1] = r
    F, R = cell.F, cell.R
    TK = Tk + 273.15
    SOCavg = zk[-1]
    SOCnAvg = cell.soc("neg", SOCavg, TK)
    SOCpAvg = cell.soc("pos", SOCavg, TK)
    k0n = cell.k0("neg", SOCnAvg, TK)
    k0p = cell.k0("pos", SOCpAvg, TK)
    i0n = k0n * _sqrt(zk[ind["Thetae"][0]] * (1 - zk[ind["Thetass0"]]) * zk[ind["Thetass0"]])
    i0p = k0p * _sqrt(zk[ind["Thetae"][-1]] * (1 - zk[ind["Thetass3"]]) * zk[ind["Thetass3"]])
    Rfn = cell.Rf("neg", SOCnAvg, TK)
    Rfp = cell.Rf("pos", SOCpAvg, TK)
    Cv = Rfp * C[ind["Ifdl3"]] - Rfn * C[ind["Ifdl0"]] + C[ind["Phie"][-1]]
    Dv = Rfp * D[ind["Ifdl3"]] - Rfn * D[ind["Ifdl0"]] + D[ind["Phie"][-1]]
    Upos = cell.Uocp("pos", zk[ind["Thetass3"]], TK)
    Uneg = cell.Uocp("neg", zk[ind["Thetass0"]], TK)
    If0, If3 = zk[ind["If0"]], zk[ind["If3"]]
    negEta0 = 2 * R * TK / F * math.asinh(If0 / (2 * i0n))
    posEta3 = 2 * R * TK / F * math.asinh(If3 / (2 * i0p))
    b_phi = 0.01 * 0
    bv = (Upos - Uneg) + (posEta3 - negEta0) + b_phi
    Uocpn = cell.Uocp("neg", SOCnAvg)                           # one argument (EKFmatsHandler.m:96)
    r2 = ind["negPhise"][1]
    return dict(a=a, Csoc=Csoc, Dsoc=0.0, Cv=np.concatenate([Cv, [0.0]]), Dv=Dv,
                Cphi=np.concatenate([C[r2], [0.0]]), Dphi=D[r2], bv=bv, bphi=Uocpn,
                imax=imax), xhat


# ---------------------------------------------------------------------------
# predMat / constraintsMPC / hildreth / iterMPC / initMPC
# ---------------------------------------------------------------------------
def pred_mat(a, C, D, Np, Nc):
    """predMat.m:11-53 with A = diag(a), B = ones (m = q = 1)."""
    Np = max(1, round(Np))
    Nc = max(1, min(round(Nc), Np))
    nx = len(a)
    A = np.diag(a)
    B = np.ones((nx, 1))
    Abar = np.zeros((nx + 1, nx + 1))
    Abar[:nx, :nx] = A
    Abar[:nx, nx:] = B
    Abar[nx, nx] = 1.0
    Bbar = np.zeros((nx + 1, 1))
    Bbar[nx, 0] = 1.0
    Cbar = np.concatenate([np.asarray(C, dtype=float), [float(D)]])[None, :]
    Phi = np.zeros((Np, nx + 1))
    G = np.zeros((Np, Nc))
    H = []
    X = Bbar
    for k in range(Np):
        H.append(mm(Cbar, X)[0, 0])
        X = mm(Abar, X)
    Ap = np.eye(nx + 1)
    for i in range(Np):
        Ap = mm(Abar, Ap)
        Phi[i] = mm(Cbar, Ap)[0]
        for j in range(min(i + 1, Nc)):
            G[i, j] = H[i - j]
    return Phi, G


def init_mpc(rom, SOC0, Np, Nc, targetSOC, cfg):
    """initMPC.m:29-74."""
    Np = max(1, round(Np))
    Nc = max(1, min(round(Nc), Np))
    return dict(Np=Np, Nc=Nc, Ts=cfg.get("Ts", 1.0), ref=targetSOC, maxHild=100,
                lam=None, uk_1=0.0, SOCk_1=0.0, SOC0=SOC0,
                u_max=cfg["u_max"], u_min=-rom.Q * cfg["Crate"], du_min=cfg["du_min"],
                du_max=cfg["du_max"], v_max=cfg["v_max"], phise_min=cfg["phise_min"],
                z_max=cfg["z_max"], z_tol=cfg["z_tol"], cons=cfg.get("constraints", (1, 1, 1)))


def constraints_mpc(x, MPC, mpc, Phi_s, G_s):
    """constraintsMPC.m:11-112 (terminal row off, as in runMPC)."""
    Nc, Np = mpc["Nc"], mpc["Np"]
    Ms, gs = [], []
    cu, cv, ce = mpc["cons"]
    if cu:
        Cu = np.tril(np.ones((Nc, Nc)))
        uk = mpc["uk_1"]
        Ms += [Cu, -Cu, np.eye(Nc), -np.eye(Nc)]
        gs += [(mpc["u_max"] - uk) * np.ones(Nc), -(mpc["u_min"] - uk) * np.ones(Nc),
               mpc["du_max"] * np.ones(Nc), -mpc["du_min"] * np.ones(Nc)]
    if cv:
        Phi_v, G_v = pred_mat(MPC["a"], MPC["Cv"], MPC["Dv"], Np, Nc)
        rhs_v = mv(Phi_v, x) + MPC["bv"] * np.ones(Np)
        Ms.append(G_v)
        gs.append(mpc["v_max"] * np.ones(Np) - rhs_v)
    if ce:
        Phi_e, G_e = pred_mat(MPC["a"], MPC["Cphi"], MPC["Dphi"], Np, Nc)
        rhs_e = mv(Phi_e, x) + MPC["bphi"] * np.ones(Np)
        Ms.append(-G_e)
        gs.append(-(mpc["phise_min"] * np.ones(Np)) + rhs_e)
    rhs_s = mv(Phi_s, x) + mpc["SOCk_1"] * np.ones(Np)
    zmax = mpc["z_max"] + mpc["z_tol"]
    Ms.append(G_s)
    gs.append(zmax * np.ones(Np) - rhs_s)
    return np.vstack(Ms), np.concatenate(gs)


def hildreth(E, F, M, gamma, lam0, maxIter, tol=1e-6, recip=False):
    """hildreth.m:1-46 (dense H, Gauss-Seidel dual coordinate ascent).  recip (test
    infrastructure, tools/make_golden.py's ulp ensembles): the row update as
    lambda_i - t_i * (1/H_ii), an ulp-level implementation variant of hildreth.m:35."""
    nC = M.shape[0]
    lam = np.zeros(nC) if lam0 is None else np.array(lam0, dtype=float)
    X = mldivide_spd(E, M.T)                                    # E\M'
    H = mm(M, X)
    K = mv(M, mldivide_spd(E, F)) + gamma
    k = 0
    for k in range(1, maxIter + 1):
        lam_old = lam.copy()
        for i in range(nC):
            s = 0.0
            for j in range(nC):
                s = s + H[i, j] * lam[j]
            if recip:
                w = lam[i] - (K[i] + s) * (1.0 / H[i, i])
            else:
                w = -(K[i] + s - H[i, i] * lam[i]) / H[i, i]
            lam[i] = w if w > 0 else 0.0
        d = lam - lam_old
        conv = True
        for v in d:
            if not (abs(v) < tol):
                conv = False
                break
        if conv:
            break
    rhs = F + mv(M.T, lam)
    DU = lu_solve(-E, rhs)
    return DU, lam, k


def iter_mpc(xk, MPC, mpc, smin=None):
    """iterMPC.m:17-95.  Returns (uk, info)."""
    Np, Nc = mpc["Np"], mpc["Nc"]
    uk_1 = mpc["uk_1"]
    Ref = mpc["ref"] * np.ones(Np)
    dx = np.concatenate([xk, [uk_1]])
    Phi_soc, G_soc = pred_mat(MPC["a"], MPC["Csoc"], MPC["Dsoc"], Np, Nc)
    t = mv(Phi_soc, dx)
    e = Ref - t
    F = mv((-2 * G_soc).T, e)
    GtG = mm(G_soc.T, G_soc)
    if smin is None:
        smin = np.linalg.svd(GtG, compute_uv=False)[-1]
    nF = math.sqrt(dot(F, F))
    Ru = (nF / (2 * mpc["du_max"] * math.sqrt(Nc))) - smin
    E = 2 * (GtG + Ru * np.eye(Nc))
    DU = lu_solve(-E, F)
    r = e - mv(G_soc, DU)
    J_unc = dot(r, r) + dot(mv(Ru * np.eye(Nc), DU), DU)
    # iterMPC.m:53-60 stability analysis: Kmpc = first row of E\(G_soc'*Phi_soc),
    # CL = Abar - Bbar*Kmpc (predMat.m's augmentation, A = diag(a), B = ones),
    # poles = eig(CL), sv = svd(CL) (LAPACK through numpy, as MATLAB's eig/svd)
    Kmpc = mldivide_spd(E, mm(G_soc.T, Phi_soc))[0]
    na = len(MPC["a"]) + 1
    CL = np.zeros((na, na))
    CL[:na - 1, :na - 1] = np.diag(MPC["a"])
    CL[:na - 1, na - 1] = 1.0
    CL[na - 1, na - 1] = 1.0
    CL[na - 1, :] -= Kmpc
    poles = np.linalg.eigvals(CL)
    sv = np.linalg.svd(CL, compute_uv=False)
    M, gamma = constraints_mpc(dx, MPC, mpc, Phi_soc, G_soc)
    viol = mv(M, DU) - gamma
    nexec = 0
    if np.sum(viol > 0) > 0:
        DU, lam, nexec = hildreth(E, F, M, gamma, mpc["lam"], mpc["maxHild"], recip=bool(mpc.get("hild_recip")))
        mpc["lam"] = lam
    uk = DU[0] + mpc["uk_1"]
    mpc["uk_1"] = uk
    vres = mv(M, DU) - gamma
    nviol = int(np.sum(vres > 1e-9))
    r = e - mv(G_soc, DU)
    J_fin = dot(r, r) + dot(mv(Ru * np.eye(Nc), DU), DU)
    return uk, dict(nexec=nexec, nviol=nviol, J_unc=J_unc, J_fin=J_fin, DU=DU, M=M, gamma=gamma,
                    E=E, F=F, Kmpc=Kmpc, CL=CL, poles=poles, sv=sv)


# ---------------------------------------------------------------------------
# runMPC (runMPC.m:1-112)
# ---------------------------------------------------------------------------
RUNMPC_DEFAULTS = dict(Ts=1.0, SigmaV=1e-3, SigmaW=1e2, Np=5, Nc=2, targetSOC=95.0, Crate=2.0,
                       u_max=2.0, du_min=-50.0, du_max=50.0, v_min=3.4, v_max=4.1,
                       phise_min=0.08, z_max=0.95, z_tol=0.0, constraints=(1, 1, 1))


def run_cell(rom, SOC0, TC, nsteps, cfg=None, record_state=False, tc_traj=None):
    """Closed loop for ONE cell (runMPC.m:72-112).  Returns dict of trajectories.
    tc_traj [nsteps] (degC): the temperature passed to OB_step / iterEKF / EKFmatsHandler
    at each step (runMPC.m:85-92 passes TC); TC is the initial one (initKF, first OB_step)."""
    with np.errstate(all="ignore"):
        return _run_cell(rom, SOC0, TC, nsteps, cfg, record_state, tc_traj)


def _run_cell(rom, SOC0, TC, nsteps, cfg, record_state, tc_traj=None):
    c = dict(RUNMPC_DEFAULTS)
    if cfg:
        c.update(cfg)
    SigmaX0 = np.diag([1.0] * rom.n + [2e6])
    hm = bool(c.get("handles", False))   # cellData.function handles called directly (Cell)
    ekf = init_kf(rom, SOC0, TC, SigmaX0, c["SigmaV"], c["SigmaW"], c.get("method", "OB"), hm)
    mpc = init_mpc(rom, SOC0, c["Np"], c["Nc"], c["targetSOC"], c)
    cs = ob_step_init(rom, SOC0, TC, hm)
    mpc["hild_recip"] = bool(c.get("hild_recip", False))   # test infrastructure (ulp ensembles)
    uk = 0.0
    ob_step(uk, TC, cs)                                         # runMPC.m:74 (state no-op)
    nz = rom.nz
    out = {k: np.full(nsteps, NAN) for k in ("u", "v", "soc", "phise")}
    out["nexec"] = np.zeros(nsteps, dtype=np.int64)
    out["zk"] = np.full((nsteps, nz + 2), NAN)
    out["zbk"] = np.full((nsteps, nz + 2), NAN)
    out["status"] = np.zeros(nsteps, dtype=np.int64)
    out["poles"] = np.full((nsteps, 7), NAN + 0j)
    out["sv"] = np.full((nsteps, 7), NAN)
    out["CL"] = np.full((nsteps, 7, 7), NAN)
    # test infrastructure (tools/make_golden.py make_envelopes): cfg["ulp_kick"] = (seed, K)
    # moves each step's command by a random -K..K ulps, a stand-in for the ulp-level
    # differences between implementations of the same arithmetic (BLAS order, libm)
    kick = c.get("ulp_kick")
    krng = np.random.Generator(np.random.PCG64(kick[0])) if kick else None
    for k in range(nsteps):
        if tc_traj is not None:
            TC = float(tc_traj[k])
        V = ob_step(uk, TC, cs)
        zk, zbk, Xind = iter_ekf(ekf, V, uk, TC)
        if ekf["status"] & ST_ERROR:
            out["status"][k] = ekf["status"]
            uk = NAN
            continue
        MPC, xhat = ekf_mats_handler(ekf, Xind, zk, TC)
        phise = dot(MPC["Cphi"], xhat) + uk * MPC["Dphi"] + MPC["bphi"]
        mpc["SOCk_1"] = zk[-1]
        uk, info = iter_mpc(xhat, MPC, mpc)
        if krng is not None and np.isfinite(uk):
            steps = int(krng.integers(-kick[1], kick[1] + 1))
            for _ in range(abs(steps)):
                uk = float(np.nextafter(uk, np.inf if steps > 0 else -np.inf))
            mpc["uk_1"] = uk
        out["u"][k] = uk
        out["v"][k] = V
        out["soc"][k] = zk[-1]
        out["phise"][k] = phise
        out["nexec"][k] = info["nexec"]
        out["zk"][k] = zk
        out["zbk"][k] = zbk
        out["status"][k] = ekf["status"]
        out["poles"][k] = info["poles"]
        out["sv"][k] = info["sv"]
        out["CL"][k] = info["CL"]
    if record_state:
        out["ekf"] = ekf
        out["mpc"] = mpc
        out["cs"] = cs
    return out
