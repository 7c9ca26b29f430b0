"""ROM container, synthetic NMC30-like ROM generator and device packing.

The reference loads ``ROM_NMC30_HRA.mat`` (runMPC.m:4-5).  That file is listed in
the reference's ``.MISSING_LARGE_BLOBS:1`` and is absent, and it also carries the
``cellData.function.*`` MATLAB handles the hot path calls (OB_step.m:203-219,
iterEKF.m:282-283,362-363,392-407, EKFmatsHandler.m:53-92).  This module

* defines :class:`ROM`, a plain-array mirror of the MATLAB ``ROM`` struct
  (``ROMmdls(T,Z).{A,B,C,D,T,SOC}``, ``tfData.{names,xLoc}``,
  ``xraData.{T,SOC,Tsamp}``, ``cellData``);
* defines the *tabulated* ``cellData.function`` semantics this framework uses
  (every handle of (theta, T) as a [ntemp, ntheta] table with a defined bilinear
  lookup, ``soc(z, T)`` from its z = 0 / 1 ends), identical in the numpy oracle, the
  C oracle and the HIP kernels;
* generates a deterministic synthetic NMC30-like ROM (3 x 21 set-points, n = 5,
  nz = 26 outputs) that satisfies every index check of iterEKF.m:692-734 and
  OB_step.m:140-158;
* resolves the output-row roles (iterEKF.m:610-735) and packs everything into
  the flat arrays the C-ABI ``mpcekf_rom`` struct expects (include/mpcekf.h).

A real ROM is exported on a MATLAB machine by ``matlab/mpcekf_export_rom.m`` (it
tabulates the cellData handles) and loaded with :func:`ROM.load_json` (SURVEY.md
§8(f) rank 1); :func:`ROM.load_npz` reads this module's own ``save_npz`` files.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# --------------------------------------------------------------------------
# tfData name codes (shared with include/mpcekf.h: MPCEKF_TF_*)
# --------------------------------------------------------------------------
TF_NAMES = [
    "negIfdl", "posIfdl", "negIf", "posIf", "negIdl", "posIdl",
    "negPhis", "posPhis", "negPhise", "posPhise", "negThetass", "posThetass",
    "negPhie", "sepPhie", "posPhie", "negThetae", "sepThetae", "posThetae",
]
TF_CODE = {n: i for i, n in enumerate(TF_NAMES)}

# Role slots: the 11 rows the hot path addresses individually.  The device
# layout puts them first, in this order (see DESIGN.md "row permutation").
ROLE_NAMES = ["Ifdl0", "Ifdl3", "If0", "If3", "Thetass0", "Thetass3",
              "Thetae1", "Thetae_end", "Phie_end", "Phise0", "negPhise2"]
NROLE = len(ROLE_NAMES)

# per-row group flags (include/mpcekf.h: MPCEKF_G_*)
G_NEG_THETASS = 1 << 0
G_POS_THETASS = 1 << 1
G_NEG_PHISE = 1 << 2
G_POS_PHISE = 1 << 3
G_PHIE = 1 << 4          # member of ind.Phie (after the loc==0 drop)
G_PHIE_LOC0 = 1 << 5     # member of ind.Phie with loc == 0 (iterEKF.m:374-375)
G_THETAE = 1 << 6
G_POS_PHIS = 1 << 7

# getChatZ Chat0 kinds (iterEKF.m:540-586), last assignment wins
C0_ZERO, C0_CHATV0, C0_RES0N, C0_RES0P, C0_DUN_RES0N, C0_DUP_RES0P, C0_MDUN_RES0N = range(7)

EPS = np.finfo(float).eps


EL_TABLES = ("Uocp", "dUocp", "k0", "Rf", "Cdleff")   # [ntemp, ntheta] each (include/mpcekf.h)


@dataclass
class Electrode:
    """One electrode's ``cellData.function.{neg,pos}`` handles, tabulated on the ROM's
    (T, theta) grid (:attr:`ROM.tab_T_K` x uniform theta over [0, 1]).

    ABI v3 (optional): ``poly`` holds, per table, the coefficients of a piecewise
    polynomial in theta ([ntemp, ntheta - 1, npoly], ``Uocp1``: [ntheta - 1, npoly];
    npoly 4: cubic, 6: quintic Hermite); when present the lookups use them instead of
    the linear interpolation of the node values.  ``Ea``
    gives a function an Arrhenius factor exp(Ea/R (1/Tref - 1/T)) applied after the
    temperature interpolation of its rows (0: none).  See :func:`eval_fn`."""
    theta0: float              # theta0(): the plant's zero-argument call (OB_step.m:207-210)
    theta100: float            # theta100()
    soc0: np.ndarray           # [ntemp] soc(0, T)
    soc100: np.ndarray         # [ntemp] soc(1, T)
    Uocp: np.ndarray           # [ntemp, ntheta] Uocp(theta, T)
    Uocp1: np.ndarray          # [ntheta] Uocp(theta), the one-argument call (EKFmatsHandler.m:96)
    dUocp: np.ndarray          # [ntemp, ntheta] dUocp(theta, T)
    k0: np.ndarray             # [ntemp, ntheta] k0(theta, T)
    Rf: np.ndarray             # [ntemp, ntheta] Rf(theta, T)
    Cdleff: np.ndarray         # [ntemp, ntheta] Cdl^(2-nDL) wDL^(nDL-1) (OB_step.m:212-219)
    poly: dict = None          # ABI v3: {"Uocp": [ntemp, ntheta-1, npoly], ..., "Uocp1": [ntheta-1, npoly]}
    Ea: dict = None            # ABI v3: {"k0": J/mol, ...}; missing / 0: no Arrhenius factor
    # ABI v4: functions on their own theta nodes, {"Uocp": (x [m], coef [ntemp, m-1, npoly]), ...,
    # "Uocp1": (x, coef [m-1, npoly])}; a function named here is looked up by interp_nodes
    # instead of its uniform-grid poly (which may then be absent)
    nodes: dict = None


def interp_tab(tab: np.ndarray, x: float) -> float:
    """Piecewise-linear table lookup on a uniform grid over [0, 1].

    NaN in -> NaN out; the abscissa is clamped to [0, 1].  The C oracle
    (oracle/mpcekf_oracle.c: tab_interp) and the kernels (csrc: tabi)
    evaluate exactly this expression sequence.
    """
    if x != x:
        return float("nan")
    n = tab.shape[0]
    xc = min(max(x, 0.0), 1.0)
    t = xc * (n - 1)
    i = int(math.floor(t))
    if i > n - 2:
        i = n - 2
    f = t - i
    return float(tab[i] + f * (tab[i + 1] - tab[i]))


def interp_poly(coef: np.ndarray, x: float) -> float:
    """ABI v3 piecewise-polynomial lookup: coef [ntheta - 1, npoly] over the uniform theta
    grid of ntheta nodes.  The interval i and its local s = t - i are found as in
    :func:`interp_tab`; the value is Horner's c0 + s (c1 + s (... + s c_last)) (no
    contraction).  The library evaluates 6 coefficients, a cubic's two upper ones zero,
    which gives the same value.  Same sequence in the C oracle (tab_poly) and the kernels
    (tabp)."""
    if x != x:
        return float("nan")
    n = coef.shape[0] + 1
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


def node_segment(x: np.ndarray, th: float):
    """ABI v4 segment of theta on a function's own nodes x [m] (strictly ascending): theta
    clamped to [0, 1], k = #{j in 1..m-2 : x_j <= theta} (the segment holding it, segments 0
    and m-2 extended past the end nodes), s = theta - x_k.  The C oracle (node_seg) states
    the same; the kernels find k through a uniform bucket map (host build_rom) that gives
    this k exactly."""
    xc = min(max(th, 0.0), 1.0)
    k = int(np.searchsorted(x[1:-1], xc, side="right"))
    return k, xc - float(x[k])


def interp_nodes(x: np.ndarray, coef: np.ndarray, th: float) -> float:
    """ABI v4 row: segment k's polynomial in s = theta - x_k (coef [m-1, npoly]), Horner
    c0 + s (c1 + s (... + s c_last)) (no contraction; the C oracle and kernels: fma).  An
    interp1-linear handle's segment is (y_k, slope_k, 0, 0): y_k + s slope_k, np.interp's
    value to the last bit up to its separate rounding of the product."""
    if th != th:
        return float("nan")
    k, s = node_segment(x, th)
    c = coef[k]
    v = float(c[-1])
    for j in range(len(c) - 2, -1, -1):
        v = float(c[j] + s * v)
    return v


# Defined exp (the Arrhenius factor of the v3 lookup): fdlibm's reduction x = k ln2 + r and
# its rational remez form, with only correctly rounded operations, so the kernels (dexp),
# the C oracle (orc_exp) and this function give the same bits.
_EXP_P = (1.66666666666666019037e-01, -2.77777777770155933842e-03, 6.61375632143793436117e-05,
          -1.65339022054652515390e-06, 4.13813679705723846039e-08)
_LN2_HI, _LN2_LO, _INVLN2 = 6.93147180369123816490e-01, 1.90821492927058770002e-10, 1.44269504088896338700e+00


def dexp(x: float) -> float:
    if x != x:
        return x
    if x > 709.782712893384:
        return math.inf
    if x < -745.1332191019412:
        return 0.0
    k = math.floor(x * _INVLN2 + 0.5)
    hi = x - k * _LN2_HI
    lo = k * _LN2_LO
    r = hi - lo
    t = r * r
    P1, P2, P3, P4, P5 = _EXP_P
    c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))))
    y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi)
    return math.ldexp(y, int(k))


def arrhenius(Ea_over_R: float, Tref: float, T: float) -> float:
    """The v3 Arrhenius factor exp(Ea/R (1/Tref - 1/T)), spelled as the kernels do."""
    return dexp(Ea_over_R * (1.0 / Tref - 1.0 / T))


def temp_index(T_K: np.ndarray, T: float):
    """(j, g) of T on the table temperature grid: T clamped to the grid ends, j the
    last grid index with T_K[j] <= T (at most ntemp - 2), g = (T - T_K[j]) / (T_K[j+1] - T_K[j]).
    A single-point grid gives (0, 0.0).  Same sequence in the kernels and the C oracle."""
    nt = len(T_K)
    if nt == 1:
        return 0, 0.0
    Tc = min(max(T, float(T_K[0])), float(T_K[-1]))
    j = 0
    while j < nt - 2 and Tc >= T_K[j + 1]:
        j += 1
    return j, float((Tc - T_K[j]) / (T_K[j + 1] - T_K[j]))


def eval_tab2(tab2: np.ndarray, theta: float, jg, coef=None, nodes=None) -> float:
    """Defined bilinear lookup of a [ntemp, ntheta] table: the theta interpolation of rows
    j and j+1, then a + g (b - a).  coef [ntemp, ntheta-1, 4] (ABI v3): the rows are the
    piecewise polynomials instead of the linear interpolation of tab2; nodes (x, coef
    [ntemp, m-1, npoly]) (ABI v4): the rows are polynomials on the function's own nodes."""
    j, g = jg
    if nodes is not None:
        x, cn = nodes
        row = lambda k: interp_nodes(x, cn[k], theta)
    elif coef is None:
        row = lambda k: interp_tab(tab2[k], theta)
    else:
        row = lambda k: interp_poly(coef[k], theta)
    a = row(j)
    if tab2.shape[0] == 1:
        return a
    b = row(j + 1)
    return float(a + g * (b - a))


def eval_fn(e: Electrode, name: str, theta: float, jg, T: float, R: float, Tref: float) -> float:
    """The v3 lookup of one cellData.function handle (include/mpcekf.h): the rows of
    ``name`` at theta (polynomial when ``e.poly`` has them, else linear), linear in T between
    the bracketing rows, times the Arrhenius factor when ``e.Ea[name]`` is non-zero."""
    v = eval_tab2(getattr(e, name), theta, jg, None if not e.poly else e.poly.get(name),
                  None if not e.nodes else e.nodes.get(name))
    ea = 0.0 if not e.Ea else float(e.Ea.get(name, 0.0))
    if ea != 0.0:
        v = v * arrhenius(ea / R, Tref, T)
    return v


def eval_tab1(tab1: np.ndarray, jg) -> float:
    """A [ntemp] table at (j, g): tab[j] + g (tab[j+1] - tab[j])."""
    j, g = jg
    if tab1.shape[0] == 1:
        return float(tab1[0])
    return float(tab1[j] + g * (tab1[j + 1] - tab1[j]))


class CellFunctions:
    """The tabulated ``cellData.function.{neg,pos}`` handles of one electrode."""

    def __init__(self, e: Electrode, T_K: np.ndarray, R: float = 8.3144621, Tref: float = 298.15):
        self.e = e
        self.T_K = np.asarray(T_K, dtype=float)
        self.R, self.Tref = R, Tref

    def soc(self, z, T):                      # cellData.function.neg.soc(z,T)
        jg = temp_index(self.T_K, T)
        s0, s1 = eval_tab1(self.e.soc0, jg), eval_tab1(self.e.soc100, jg)
        return s0 + z * (s1 - s0)

    def _f(self, name, theta, T):
        return eval_fn(self.e, name, theta, temp_index(self.T_K, T), T, self.R, self.Tref)

    def Uocp(self, theta, T=None):            # 1-arg call: its own table (EKFmatsHandler.m:96)
        if T is None:
            if self.e.nodes and "Uocp1" in self.e.nodes:
                return interp_nodes(*self.e.nodes["Uocp1"], theta)
            if self.e.poly:
                return interp_poly(self.e.poly["Uocp1"], theta)
            return interp_tab(self.e.Uocp1, theta)
        return self._f("Uocp", theta, T)

    def dUocp(self, theta, T):
        return self._f("dUocp", theta, T)

    def k0(self, theta, T):
        return self._f("k0", theta, T)

    def Rf(self, theta, T):
        return self._f("Rf", theta, T)

    def Cdleff(self, theta, T):
        return self._f("Cdleff", theta, T)

    def theta0(self):
        return self.e.theta0

    def theta100(self):
        return self.e.theta100


@dataclass
class ROM:
    """Plain-array mirror of the MATLAB ROM struct (runMPC.m:5)."""
    T_degC: np.ndarray         # xraData.T  [nT] (ascending)
    SOC_pct: np.ndarray        # xraData.SOC [nZ] (ascending)
    Ts: float                  # xraData.Tsamp
    A: np.ndarray              # [nT, nZ, n+1] diag(ROMmdls(t,z).A), last == 1
    C: np.ndarray              # [nT, nZ, nz, n+1]
    D: np.ndarray              # [nT, nZ, nz]
    names: list                # tfData.names [nz]
    xloc: np.ndarray           # tfData.xLoc [nz]
    F: float
    R: float
    Q: float                   # cellData.function.const.Q(), Ah
    Rc: float
    Tref: float
    tab_T_K: np.ndarray        # [ntemp] temperature grid of the electrode tables (K, ascending)
    neg: Electrode
    pos: Electrode
    meta: dict = field(default_factory=dict)

    # ---- shapes -------------------------------------------------------
    @property
    def nT(self):
        return self.A.shape[0]

    @property
    def nZ(self):
        return self.A.shape[1]

    @property
    def n(self):
        return self.A.shape[2] - 1

    @property
    def nz(self):
        return self.C.shape[2]

    @property
    def NM(self):
        return self.nT * self.nZ

    def fn(self, which):
        return CellFunctions(self.neg if which == "neg" else self.pos, self.tab_T_K, self.R, self.Tref)

    @property
    def npoly(self):
        """ABI v3: coefficients per theta interval of the electrode tables (4 cubic, 6
        quintic), 0 for v2 linear tables.  With ABI v4 nodes the largest of the uniform-grid
        and node polynomials (the library pads each to 6)."""
        n = 0
        for e in (self.neg, self.pos):
            for c in (e.poly or {}).values():
                n = max(n, int(np.asarray(c).shape[-1]))
            for _, c in (e.nodes or {}).values():
                n = max(n, int(np.asarray(c).shape[-1]))
        return n

    @property
    def ntheta(self):
        return int(self.neg.Uocp.shape[1])

    @property
    def ntemp(self):
        return int(np.asarray(self.tab_T_K).size)

    # ROMmdls(t,z).T / .SOC exactly as initKF.m:57-59 reads them
    def mdl_T_K(self):
        return np.array([self.T_degC[t] + 273.15 for t in range(self.nT)])

    def mdl_Z(self):
        return np.array([self.SOC_pct[z] / 100 for z in range(self.nZ)])

    # ---- index resolution (iterEKF.m:610-735, OB_step.m:86-163) --------
    def resolve_indices(self):
        names = list(self.names)
        loc = np.asarray(self.xloc, dtype=float)

        def find(nm):
            return [i for i, s in enumerate(names) if s == nm]

        ind = {nm: find(nm) for nm in TF_NAMES}
        Ifdl = ind["negIfdl"] + ind["posIfdl"]
        If = ind["negIf"] + ind["posIf"]
        Thetass = ind["negThetass"] + ind["posThetass"]
        Phise = ind["negPhise"] + ind["posPhise"]
        Phie = ind["negPhie"] + ind["sepPhie"] + ind["posPhie"]
        Thetae = ind["negThetae"] + ind["sepThetae"] + ind["posThetae"]

        def at(lst, x):
            return [i for i in lst if loc[i] == x]

        r = {}
        r["Ifdl0"], r["Ifdl3"] = at(Ifdl, 0), at(Ifdl, 3)
        r["If0"], r["If3"] = at(If, 0), at(If, 3)
        r["Thetass0"], r["Thetass3"] = at(Thetass, 0), at(Thetass, 3)
        r["Phise0"] = at(Phise, 0)
        for k in ("Ifdl0", "Ifdl3", "If0", "If3", "Thetass0", "Thetass3", "Phise0"):
            if len(r[k]) != 1:
                raise ValueError(f"ROM must have exactly one {k} output (iterEKF.m:692-725); got {r[k]}")
        if not Thetae or loc[Thetae[0]] > 0:
            raise ValueError("Simulation requires thetae at negative-collector! (iterEKF.m:709)")
        if loc[Thetae[-1]] > 3 + EPS or loc[Thetae[-1]] < 3 - EPS:
            raise ValueError("Simulation requires thetae at positive-collector! (iterEKF.m:711)")
        if Phie and loc[Phie[0]] == 0:       # iterEKF.m:728-731 (warning, dropped)
            Phie = Phie[1:]
        if not Phie or loc[Phie[-1]] > 3 + EPS or loc[Phie[-1]] < 3 - EPS:
            raise ValueError("Simulation requires phie at positive-collector! (iterEKF.m:732)")
        if len(ind["negPhise"]) < 2:
            raise ValueError("EKFmatsHandler.m:97 needs ind.negPhise(2)")
        # OB_step's own (stricter) lookups must land on the same rows (OB_step.m:131-137)
        ob = {
            "negIfdl0": [i for i in ind["negIfdl"] if loc[i] == 0],
            "posIfdl3": [i for i in ind["posIfdl"] if loc[i] == 3],
            "negIf0": [i for i in ind["negIf"] if loc[i] == 0],
            "posIf3": [i for i in ind["posIf"] if loc[i] == 3],
            "negThetass0": [i for i in ind["negThetass"] if loc[i] == 0],
            "posThetass3": [i for i in ind["posThetass"] if loc[i] == 3],
        }
        pairs = [("negIfdl0", "Ifdl0"), ("posIfdl3", "Ifdl3"), ("negIf0", "If0"),
                 ("posIf3", "If3"), ("negThetass0", "Thetass0"), ("posThetass3", "Thetass3")]
        for a, b in pairs:
            if ob[a] != r[b]:
                raise ValueError(f"OB_step {a} and iterEKF {b} resolve to different rows")
        roles = {k: r[k][0] for k in ("Ifdl0", "Ifdl3", "If0", "If3", "Thetass0", "Thetass3", "Phise0")}
        roles["Thetae1"] = Thetae[0]
        roles["Thetae_end"] = Thetae[-1]
        roles["Phie_end"] = Phie[-1]
        roles["negPhise2"] = ind["negPhise"][1]
        rows = [roles[k] for k in ROLE_NAMES]
        if len(set(rows)) != NROLE:
            raise ValueError("role rows must be distinct for the device row permutation")
        return dict(ind=ind, Ifdl=Ifdl, If=If, Thetass=Thetass, Phise=Phise, Phie=Phie,
                    Thetae=Thetae, roles=roles, loc=loc)

    def validate(self):
        """initKF.m:66-91 structure checks plus grid ordering and table shapes."""
        if np.any(np.diff(self.T_degC) <= 0) or np.any(np.diff(self.SOC_pct) <= 0):
            raise ValueError("ROM set-points must be strictly ascending")
        tk = np.asarray(self.tab_T_K, dtype=float)
        if tk.ndim != 1 or tk.size < 1 or np.any(np.diff(tk) <= 0):
            raise ValueError("electrode table temperatures must be strictly ascending")
        for e in (self.neg, self.pos):
            for k in EL_TABLES:
                t = getattr(e, k)
                if t.ndim != 2 or t.shape != (tk.size, self.ntheta) or t.shape[1] < 2:
                    raise ValueError(f"electrode table {k}: shape {t.shape}, expected ({tk.size}, ntheta >= 2)")
            if e.Uocp1.shape != (self.ntheta,) or e.soc0.shape != (tk.size,) or e.soc100.shape != (tk.size,):
                raise ValueError("electrode tables Uocp1 / soc0 / soc100 have the wrong length")
            nd = e.nodes or {}
            for k, (x, c) in nd.items():
                if k not in EL_TABLES + ("Uocp1",):
                    raise ValueError(f"nodes: {k!r} is not one of {EL_TABLES + ('Uocp1',)}")
                x = np.asarray(x, dtype=float)
                if x.ndim != 1 or x.size < 2 or np.any(np.diff(x) <= 0) or not np.all(np.isfinite(x)):
                    raise ValueError(f"nodes {k}: need >= 2 strictly ascending finite theta nodes")
                if x.size > 2 and (x[1] <= 0.0 or x[-2] >= 1.0):
                    raise ValueError(f"nodes {k}: interior nodes must lie in (0, 1)")
                want = (x.size - 1,) if k == "Uocp1" else (tk.size, x.size - 1)
                if np.asarray(c).shape[:-1] != want or np.asarray(c).shape[-1] not in (4, 6):
                    raise ValueError(f"nodes {k}: coefficients {np.asarray(c).shape}, expected {want} x 4 or 6")
            if nd and not e.poly and set(nd) != set(EL_TABLES) | {"Uocp1"}:
                raise ValueError("nodes: functions without nodes need the uniform-grid poly tables")
            if e.poly:
                missing = (set(EL_TABLES) | {"Uocp1"}) - set(e.poly) - set(nd)
                if missing:
                    raise ValueError(f"poly tables: need all of {EL_TABLES + ('Uocp1',)} (or their nodes), "
                                     f"missing {sorted(missing)}")
                npoly = np.asarray(next(iter(e.poly.values()))).shape[-1]
                if npoly not in (4, 6):
                    raise ValueError(f"poly tables: {npoly} coefficients per interval (4: cubic, 6: quintic)")
                for k, c in e.poly.items():
                    want = (self.ntheta - 1, npoly) if k == "Uocp1" else (tk.size, self.ntheta - 1, npoly)
                    if np.asarray(c).shape != want:
                        raise ValueError(f"poly table {k}: shape {np.asarray(c).shape}, expected {want}")
            for k in (e.Ea or {}):
                if k not in EL_TABLES:
                    raise ValueError(f"Ea: {k!r} is not one of {EL_TABLES}")
        if bool(self.neg.poly or self.neg.nodes) != bool(self.pos.poly or self.pos.nodes):
            raise ValueError("poly tables must be given for both electrodes or neither")
        if not np.all(self.A[..., -1] == 1):
            raise ValueError("A does not have integrator state (initKF.m:74)")
        self.resolve_indices()

    # ---- device packing -------------------------------------------------
    def device_layout(self):
        """Row permutation + per-row flags for the kernels."""
        info = self.resolve_indices()
        roles = [info["roles"][k] for k in ROLE_NAMES]
        perm = roles + [i for i in range(self.nz) if i not in roles]
        loc = info["loc"]
        flags = np.zeros(self.nz, dtype=np.int32)
        c0 = np.zeros(self.nz, dtype=np.int32)
        ind = info["ind"]
        for i in ind["negThetass"]:
            flags[i] |= G_NEG_THETASS
        for i in ind["posThetass"]:
            flags[i] |= G_POS_THETASS
        for i in ind["negPhise"]:
            flags[i] |= G_NEG_PHISE
        for i in ind["posPhise"]:
            flags[i] |= G_POS_PHISE
        for i in info["Phie"]:
            flags[i] |= G_PHIE
            if loc[i] == 0:
                flags[i] |= G_PHIE_LOC0
        for i in info["Thetae"]:
            flags[i] |= G_THETAE
        for i in ind["posPhis"]:
            flags[i] |= G_POS_PHIS
        # Chat0 assignment order of getChatZ (iterEKF.m:553-586)
        for i in ind["posPhis"]:
            c0[i] = C0_CHATV0
        for i in ind["negThetass"]:
            c0[i] = C0_RES0N
        for i in ind["posThetass"]:
            c0[i] = C0_RES0P
        for i in ind["negPhise"]:
            c0[i] = C0_DUN_RES0N
        for i in ind["posPhise"]:
            c0[i] = C0_DUP_RES0P
        for i in info["Phie"]:
            c0[i] = C0_MDUN_RES0N
        # C row of Phise0 used by the Phie rows in getChatZ is role slot 9
        return dict(perm=np.array(perm, dtype=np.int32),
                    flags=flags[perm].astype(np.int32),
                    c0kind=c0[perm].astype(np.int32))

    # ---- persistence ----------------------------------------------------
    def to_npz_dict(self):
        d = dict(T_degC=self.T_degC, SOC_pct=self.SOC_pct, Ts=self.Ts, A=self.A, C=self.C, D=self.D,
                 names=np.array(self.names), xloc=self.xloc, F=self.F, R=self.R, Q=self.Q, Rc=self.Rc,
                 Tref=self.Tref, tab_T_K=self.tab_T_K)
        for side, e in (("neg", self.neg), ("pos", self.pos)):
            for k in _EL_SCALARS + _EL_ARRAYS:
                d[f"{side}_{k}"] = getattr(e, k)
            # ABI v3 fields only when present (a v2 ROM's dict, and so its hash, is unchanged)
            for k, v in (e.poly or {}).items():
                d[f"{side}_poly_{k}"] = np.asarray(v, dtype=float)
            for k, v in (e.Ea or {}).items():
                d[f"{side}_Ea_{k}"] = float(v)
            for k, (x, c) in (e.nodes or {}).items():   # ABI v4 (absent before: hashes unchanged)
                d[f"{side}_nodex_{k}"] = np.asarray(x, dtype=float)
                d[f"{side}_nodep_{k}"] = np.asarray(c, dtype=float)
        return d

    def save_npz(self, path):
        np.savez(path, **self.to_npz_dict())

    @staticmethod
    def load_npz(path):
        z = np.load(path, allow_pickle=False)

        def el(side):
            kw = {k: float(z[f"{side}_{k}"]) for k in _EL_SCALARS}
            for k in _EL_ARRAYS:
                kw[k] = np.array(z[f"{side}_{k}"], dtype=float)
            cub = {k[len(side) + 6:]: np.array(z[k], dtype=float) for k in z.files
                   if k.startswith(f"{side}_poly_")}
            ea = {k[len(side) + 4:]: float(z[k]) for k in z.files if k.startswith(f"{side}_Ea_")}
            nd = {k[len(side) + 7:]: (np.array(z[k], dtype=float), np.array(z[f"{side}_nodep_" + k[len(side) + 7:]],
                                                                           dtype=float))
                  for k in z.files if k.startswith(f"{side}_nodex_")}
            return Electrode(**kw, poly=cub or None, Ea=ea or None, nodes=nd or None)

        return ROM(T_degC=np.array(z["T_degC"], float), SOC_pct=np.array(z["SOC_pct"], float),
                   Ts=float(z["Ts"]), A=np.array(z["A"], float), C=np.array(z["C"], float),
                   D=np.array(z["D"], float), names=[str(s) for s in z["names"]],
                   xloc=np.array(z["xloc"], float), F=float(z["F"]), R=float(z["R"]),
                   Q=float(z["Q"]), Rc=float(z["Rc"]), Tref=float(z["Tref"]),
                   tab_T_K=np.array(z["tab_T_K"], float), neg=el("neg"), pos=el("pos"))


    # ---- JSON exchange format (matlab/mpcekf_export_rom.m) ------------------
    JSON_FORMAT = "mpcekf-rom-v2"
    JSON_FORMAT_V3 = "mpcekf-rom-v3"   # + per-table theta polynomials and Arrhenius energies
    JSON_FORMAT_V4 = "mpcekf-rom-v4"   # + per-function theta nodes (lookup-table handles)

    def to_json_dict(self):
        """The dict ``matlab/mpcekf_export_rom.m`` writes: every array as
        ``{"shape", "order": "F", "data"}`` (MATLAB column-major), scalars bare."""
        def arr(x):
            x = np.asarray(x, dtype=float)
            shape = list(x.shape) if x.ndim >= 2 else [1, int(x.size)]
            return {"shape": shape, "order": "F", "data": [_json_num(v) for v in x.ravel(order="F")]}

        def el(e):
            d = {k: float(getattr(e, k)) for k in _EL_SCALARS}
            d.update({k: arr(getattr(e, k)) for k in _EL_ARRAYS})
            if e.poly:   # v3: [ntemp, ntheta-1, 4] (Uocp1: [ntheta-1, 4]) column-major like the rest
                d["poly"] = {k: arr(v) for k, v in e.poly.items()}
            if e.Ea:
                d["Ea"] = {k: float(v) for k, v in e.Ea.items()}
            if e.nodes:   # v4: {"nodes": {"Uocp": {"x": [1, m], "p": [ntemp, m-1, npoly]}, ...}}
                d["nodes"] = {k: {"x": arr(x), "p": arr(c)} for k, (x, c) in e.nodes.items()}
            return d

        fmt = self.JSON_FORMAT
        if self.npoly or self.neg.Ea or self.pos.Ea:
            fmt = self.JSON_FORMAT_V3
        if self.neg.nodes or self.pos.nodes:
            fmt = self.JSON_FORMAT_V4
        return {"format": fmt, "T_degC": arr(self.T_degC), "SOC_pct": arr(self.SOC_pct),
                "Ts": float(self.Ts), "A": arr(self.A), "C": arr(self.C), "D": arr(self.D),
                "names": list(self.names), "xloc": arr(self.xloc), "F": float(self.F), "R": float(self.R),
                "Q": float(self.Q), "Rc": float(self.Rc), "Tref": float(self.Tref),
                "tab_T_K": arr(self.tab_T_K), "neg": el(self.neg), "pos": el(self.pos)}

    def save_json(self, path):
        import json
        with open(path, "w") as f:
            json.dump(self.to_json_dict(), f)

    @staticmethod
    def from_json_dict(d):
        """Inverse of :meth:`to_json_dict`; accepts what MATLAB's ``jsonencode`` makes of
        the exporter's struct (1-element arrays as bare numbers, NaN as null, a lone
        name as a string).  Raises ValueError on a wrong format tag or shape."""
        if d.get("format") not in (ROM.JSON_FORMAT, ROM.JSON_FORMAT_V3, ROM.JSON_FORMAT_V4):
            raise ValueError(f"ROM json: format {d.get('format')!r}, expected {ROM.JSON_FORMAT!r}, "
                             f"{ROM.JSON_FORMAT_V3!r} or {ROM.JSON_FORMAT_V4!r}")

        def arr(a, ndim):
            if a.get("order", "F") != "F":
                raise ValueError("ROM json: arrays must be column-major ('F')")
            data = np.array([np.nan if v is None else v for v in np.atleast_1d(a["data"])], dtype=float)
            shape = [int(v) for v in np.atleast_1d(a["shape"])]
            if int(np.prod(shape)) != data.size:
                raise ValueError(f"ROM json: shape {shape} does not hold {data.size} values")
            x = data.reshape(shape, order="F")
            if ndim == 1:
                return x.ravel(order="F")
            # MATLAB drops trailing singleton dimensions (e.g. nz = 1); restore them
            if x.ndim < ndim:
                x = x.reshape(list(x.shape) + [1] * (ndim - x.ndim), order="F")
            if x.ndim != ndim:
                raise ValueError(f"ROM json: expected {ndim}-D array, got shape {shape}")
            return x

        ntemp = arr(d["tab_T_K"], 1).size

        def el(e):
            kw = {k: float(e[k]) for k in _EL_SCALARS}
            for k in _EL_ARRAYS:
                if k in EL_TABLES:     # [ntemp, ntheta]; MATLAB drops the leading 1 of ntemp = 1
                    x = arr(e[k], 1) if ntemp == 1 else arr(e[k], 2)
                    kw[k] = x.reshape(ntemp, -1)
                else:
                    kw[k] = arr(e[k], 1)
            nth = kw["Uocp1"].size
            cub = {}
            pj = e.get("poly") or {}
            # coefficients per interval (4 cubic, 6 quintic) from any table's trailing dimension
            npoly = int(np.atleast_1d(next(iter(pj.values()))["shape"])[-1]) if pj else 0
            for k, a in pj.items():
                if k not in EL_TABLES + ("Uocp1",):
                    raise ValueError(f"ROM json: unknown poly table {k!r}")
                # F order with the leading ntemp (absent for Uocp1 or when MATLAB dropped a 1)
                x = np.array([np.nan if v is None else v for v in np.atleast_1d(a["data"])], dtype=float)
                shape = [int(v) for v in np.atleast_1d(a["shape"])]
                if int(np.prod(shape)) != x.size:
                    raise ValueError(f"ROM json: poly {k}: shape {shape} does not hold {x.size} values")
                x = x.reshape(shape, order="F")
                want = (nth - 1, npoly) if k == "Uocp1" else (ntemp, nth - 1, npoly)
                if x.size != int(np.prod(want)):
                    raise ValueError(f"ROM json: poly {k}: {x.size} values, expected {want}")
                cub[k] = x.reshape(want, order="F") if x.shape != want else x
            ea = {k: float(v) for k, v in (e.get("Ea") or {}).items()}
            nd = {}
            for k, a in (e.get("nodes") or {}).items():
                if k not in EL_TABLES + ("Uocp1",):
                    raise ValueError(f"ROM json: unknown nodes table {k!r}")
                x = arr(a["x"], 1)
                pv = np.array([np.nan if v is None else v for v in np.atleast_1d(a["p"]["data"])], dtype=float)
                shape = [int(v) for v in np.atleast_1d(a["p"]["shape"])]
                if int(np.prod(shape)) != pv.size:
                    raise ValueError(f"ROM json: nodes {k}: shape {shape} does not hold {pv.size} values")
                npn = shape[-1]
                want = (x.size - 1, npn) if k == "Uocp1" else (ntemp, x.size - 1, npn)
                if pv.size != int(np.prod(want)):
                    raise ValueError(f"ROM json: nodes {k}: {pv.size} values, expected {want}")
                pv = pv.reshape(shape, order="F")
                nd[k] = (x, pv.reshape(want, order="F") if pv.shape != want else pv)
            return Electrode(**kw, poly=cub or None, Ea=ea or None, nodes=nd or None)

        names = d["names"]
        names = [names] if isinstance(names, str) else [str(s) for s in names]
        rom = ROM(T_degC=arr(d["T_degC"], 1), SOC_pct=arr(d["SOC_pct"], 1), Ts=float(d["Ts"]),
                  A=arr(d["A"], 3), C=arr(d["C"], 4), D=arr(d["D"], 3), names=names,
                  xloc=arr(d["xloc"], 1), F=float(d["F"]), R=float(d["R"]), Q=float(d["Q"]),
                  Rc=float(d["Rc"]), Tref=float(d["Tref"]), tab_T_K=arr(d["tab_T_K"], 1),
                  neg=el(d["neg"]), pos=el(d["pos"]),
                  meta={k: d[k] for k in ("source", "tab_error") if k in d})
        nT, nZ = rom.T_degC.size, rom.SOC_pct.size
        if rom.A.shape[:2] != (nT, nZ) or rom.C.shape[:2] != (nT, nZ) or rom.D.shape[:2] != (nT, nZ):
            raise ValueError("ROM json: A/C/D set-point grid does not match xraData.T x xraData.SOC")
        if rom.C.shape[2] != len(names) or rom.D.shape[2] != len(names) or rom.xloc.size != len(names):
            raise ValueError("ROM json: C/D/xloc rows do not match tfData.names")
        return rom

    @staticmethod
    def load_json(path):
        import json
        with open(path) as f:
            return ROM.from_json_dict(json.load(f))

    @staticmethod
    def load(path):
        """Load a ROM exported by matlab/mpcekf_export_rom.m (.json) or saved by
        :meth:`save_npz` (.npz)."""
        return ROM.load_json(path) if str(path).endswith(".json") else ROM.load_npz(path)


_EL_SCALARS = ("theta0", "theta100")
_EL_ARRAYS = ("soc0", "soc100", "Uocp", "Uocp1", "dUocp", "k0", "Rf", "Cdleff")


def _json_num(v):
    v = float(v)
    return None if v != v else v   # MATLAB jsonencode writes NaN as null


# --------------------------------------------------------------------------
# Synthetic NMC30-like ROM
# --------------------------------------------------------------------------
# Output list: (tf name, xLoc, D [V or flux per A], DC gain per mode per A, res0 kind)
# Sign convention of the reference: Iapp < 0 charges (OB_step.m:7).
_M = 1.0 / 30.0   # flux normalisation: |i_f| ~ 1 at 1C
_OUTPUTS = [
    ("negIfdl", 0.0, +1.40 * _M, [-0.25 * _M, -0.10 * _M, -0.05 * _M, 0, 0], None),
    ("negIfdl", 1.0, +0.60 * _M, [+0.25 * _M, +0.10 * _M, +0.05 * _M, 0, 0], None),
    ("posIfdl", 2.0, -0.70 * _M, [-0.20 * _M, -0.10 * _M, 0, 0, 0], None),
    ("posIfdl", 3.0, -1.30 * _M, [+0.20 * _M, +0.10 * _M, 0, 0, 0], None),
    ("negIf", 0.0, +1.20 * _M, [-0.05 * _M, -0.10 * _M, -0.05 * _M, 0, 0], None),
    ("negIf", 1.0, +0.80 * _M, [+0.05 * _M, +0.10 * _M, +0.05 * _M, 0, 0], None),
    ("posIf", 2.0, -0.90 * _M, [-0.05 * _M, -0.05 * _M, 0, 0, 0], None),
    ("posIf", 3.0, -1.10 * _M, [+0.05 * _M, +0.05 * _M, 0, 0, 0], None),
    ("negIdl", 0.0, +0.20 * _M, [-0.20 * _M, 0, 0, 0, 0], None),
    ("posIdl", 3.0, -0.20 * _M, [+0.20 * _M, 0, 0, 0, 0], None),
    ("negPhis", 1.0, +2e-5, [1e-5, 0, 0, 0, 0], None),
    ("posPhis", 2.0, -1e-5, [-1e-5, 0, 0, 0, 0], None),
    ("posPhis", 3.0, -2e-5, [-1e-5, 0, 0, 0, 0], None),
    ("negPhise", 0.0, +3.0e-4, [1e-4, 1e-4, 1e-4, 1.5e-4, 5e-5], None),
    ("negPhise", 1.0, +4.0e-4, [1e-4, 1e-4, 2e-4, 2e-4, 5e-5], None),
    ("posPhise", 3.0, -3.0e-4, [-1e-4, -1e-4, -1e-4, -1e-4, 0], None),
    ("negThetass", 0.0, 0.0, [0, 0, -4e-4, -6e-4, -1e-4], "n"),
    ("negThetass", 1.0, 0.0, [0, 0, -5e-4, -7e-4, -1e-4], "n"),
    ("posThetass", 2.0, 0.0, [0, 0, 3.5e-4, 4.5e-4, 1e-4], "p"),
    ("posThetass", 3.0, 0.0, [0, 0, 3.0e-4, 4.0e-4, 1e-4], "p"),
    ("negPhie", 1.0, -1e-4, [-5e-5, -5e-5, 0, 0, 0], None),
    ("sepPhie", 1.5, -2e-4, [-1e-4, -1e-4, -5e-5, 0, 0], None),
    ("posPhie", 3.0, -4e-4, [-1e-4, -2e-4, -2e-4, 0, 0], None),
    ("negThetae", 0.0, 0.0, [0, 5e-4, 1e-3, 1e-3, 0], None),
    ("sepThetae", 1.5, 0.0, [0, 2e-4, 3e-4, 0, 0], None),
    ("posThetae", 3.0, 0.0, [0, -5e-4, -1e-3, -1e-3, 0], None),
]
_FLUX = {"negIfdl", "posIfdl", "negIf", "posIf", "negIdl", "posIdl"}
_TAU_REF = np.array([2.0, 8.0, 30.0, 120.0, 500.0])   # s at 25 degC


def _u_neg(th):
    # graphite-like: ~0.20 V at 10 % SOC, ~0.14 V at 53 %, ~0.09 V at 100 %
    return (0.088 + 0.1 * np.exp(-8 * th) + 0.03 * (1 - np.tanh((th - 0.55) / 0.12))
            + 0.4 * np.exp(-60 * th))


def _u_pos(th):
    # NMC-like: OCV(z) ~ 3.56 V at 10 %, ~4.07 V at 95 % with the graphite curve
    d = th - 0.4965
    return 4.10 - 1.31 * d + 0.9 * d * d - 0.3 * np.exp(40 * (th - 1.0)) + 0.2 * np.exp(-40 * (th - 0.35))


def _deriv(fun, th, h=1e-6):
    return (fun(th + h) - fun(th - h)) / (2 * h)


def _synth_electrode(T_K, th, Tref, R, *, theta0, theta100, u, dudt, k0ref, Ea_k0, Rf, Ea_rf, wDL, Cdl, nDL):
    """Tabulate one synthetic electrode: entropic OCP U(th) + (T - Tref) dU/dT(th) and its
    theta derivative, Arrhenius k0 with a mild theta dependence, Arrhenius film
    resistance growing with lithiation, and the double-layer Cdleff of OB_step.m:212-219
    with a small temperature coefficient."""
    dT = (T_K - Tref)[:, None]
    arr_k = np.exp(Ea_k0 / R * (1.0 / Tref - 1.0 / T_K))[:, None]
    arr_r = np.exp(Ea_rf / R * (1.0 / T_K - 1.0 / Tref))[:, None]
    cdl = Cdl * (1.0 + 2e-3 * dT)
    ones = np.ones((T_K.size, 1))
    return Electrode(theta0=theta0, theta100=theta100, soc0=np.full(T_K.size, theta0),
                     soc100=np.full(T_K.size, theta100),
                     Uocp=u(th)[None, :] + dT * dudt(th)[None, :], Uocp1=u(th),
                     dUocp=_deriv(u, th)[None, :] + dT * _deriv(dudt, th)[None, :],
                     k0=k0ref * arr_k * (0.9 + 0.4 * th * (1 - th))[None, :],
                     Rf=Rf * arr_r * (0.8 + 0.4 * th)[None, :],
                     Cdleff=(cdl ** (2 - nDL)) * (wDL ** (nDL - 1)) * ones * np.ones_like(th)[None, :])


def _du_neg(th):
    return (-0.8 * np.exp(-8 * th) - 0.25 / np.cosh((th - 0.55) / 0.12) ** 2 - 24.0 * np.exp(-60 * th))


def _d2u_neg(th):
    x = (th - 0.55) / 0.12
    return (6.4 * np.exp(-8 * th) + (2 * 0.03 / 0.12 ** 2) * np.tanh(x) / np.cosh(x) ** 2
            + 1440.0 * np.exp(-60 * th))


def _d3u_neg(th):
    x = (th - 0.55) / 0.12
    sc2 = 1.0 / np.cosh(x) ** 2
    return (-51.2 * np.exp(-8 * th) + (2 * 0.03 / 0.12 ** 3) * sc2 * (sc2 - 2 * np.tanh(x) ** 2)
            - 86400.0 * np.exp(-60 * th))


def _du_pos(th):
    return -1.31 + 1.8 * (th - 0.4965) - 12.0 * np.exp(40 * (th - 1.0)) - 8.0 * np.exp(-40 * (th - 0.35))


def _d2u_pos(th):
    return 1.8 - 480.0 * np.exp(40 * (th - 1.0)) + 320.0 * np.exp(-40 * (th - 0.35))


def _d3u_pos(th):
    return -19200.0 * np.exp(40 * (th - 1.0)) - 12800.0 * np.exp(-40 * (th - 0.35))


class SynthHandles:
    """The synthetic electrodes' ``cellData.function.{neg,pos}`` as closed-form handles:
    what a MATLAB ROM's function handles are to its exported tables.  ``make_synth_rom``
    tabulates exactly these functions (the v2 tables sample them; the v3 tables fit them
    by piecewise cubics with an exact Arrhenius factor), and ``oracle_np``'s handle mode
    (``Cell(rom, handles=True)``) calls them at every reference call site, as MATLAB
    would (OB_step.m:212-215,231-232,313-314,329-340; iterEKF.m:282-283,362-363,392-407,
    463-464,495-500,577-580; EKFmatsHandler.m:57-69,84-85,96).

    Families (Plett's parameter conventions): OCP with an entropic term,
    U(th, T) = U0(th) + (T - Tref) dU/dT(th); Arrhenius kinetics and film resistance,
    k0(th, T) = k0ref g(th) exp(Ea/R (1/Tref - 1/T)); the double-layer Cdleff of
    OB_step.m:212-219 with a linear temperature coefficient of Cdl."""

    def __init__(self, *, theta0, theta100, u, du, d2u, d3u, dudt, ddudt, d2dudt, d3dudt, k0ref, Ea_k0, Rf, Ea_rf,
                 wDL, Cdl, nDL, R, Tref):
        self.th0, self.th100 = theta0, theta100
        self.u, self.du, self.d2u, self.d3u = u, du, d2u, d3u
        self.dudt, self.ddudt, self.d2dudt, self.d3dudt = dudt, ddudt, d2dudt, d3dudt
        self.k0ref, self.Ea_k0, self.Rf0, self.Ea_rf = k0ref, Ea_k0, Rf, Ea_rf
        self.wDL, self.Cdl, self.nDL = wDL, Cdl, nDL
        self.R, self.Tref = R, Tref

    # zero-argument calls (OB_step.m:207-210)
    def theta0(self):
        return self.th0

    def theta100(self):
        return self.th100

    def soc(self, z, T):
        return self.th0 + z * (self.th100 - self.th0)

    def Uocp(self, th, T=None):
        if T is None:                      # one argument (EKFmatsHandler.m:96): the Tref curve
            return float(self.u(th))
        return float(self.u(th) + (T - self.Tref) * self.dudt(th))

    def dUocp(self, th, T):
        return float(self.du(th) + (T - self.Tref) * self.ddudt(th))

    def _arr(self, Ea, T):
        return math.exp(Ea / self.R * (1.0 / self.Tref - 1.0 / T))

    def k0(self, th, T):
        return float(self.k0ref * self._arr(self.Ea_k0, T) * (0.9 + 0.4 * th * (1 - th)))

    def Rf(self, th, T):
        return float(self.Rf0 * self._arr(-self.Ea_rf, T) * (0.8 + 0.4 * th))

    def Cdleff(self, th, T):
        cdl = self.Cdl * (1.0 + 2e-3 * (T - self.Tref))
        return float((cdl ** (2 - self.nDL)) * (self.wDL ** (self.nDL - 1)))

    # ---- tabulation: values and theta-slopes on arrays, per function --------------------
    def rows(self, name, th, T):
        """(value, d/dtheta, d2/dtheta2) of ``name`` at the theta array and temperature T
        (K), with the Arrhenius factor divided out for the functions :meth:`energies` names."""
        one = np.ones_like(th)
        dT = T - self.Tref
        if name == "Uocp":
            return (self.u(th) + dT * self.dudt(th), self.du(th) + dT * self.ddudt(th),
                    self.d2u(th) + dT * self.d2dudt(th))
        if name == "dUocp":
            return (self.du(th) + dT * self.ddudt(th), self.d2u(th) + dT * self.d2dudt(th),
                    self.d3u(th) + dT * self.d3dudt(th))
        if name == "k0":
            return self.k0ref * (0.9 + 0.4 * th * (1 - th)), self.k0ref * 0.4 * (1 - 2 * th), -0.8 * self.k0ref * one
        if name == "Rf":
            return self.Rf0 * (0.8 + 0.4 * th), self.Rf0 * 0.4 * one, 0.0 * one
        if name == "Cdleff":
            return self.Cdleff(0.0, T) * one, 0.0 * one, 0.0 * one
        if name == "Uocp1":
            return self.u(th), self.du(th), self.d2u(th)
        raise KeyError(name)

    def energies(self):
        """Ea (J/mol) of the v3 Arrhenius factor per function (Rf falls with T: -Ea)."""
        return {"k0": self.Ea_k0, "Rf": -self.Ea_rf}


def hermite_coefs(y, m, h, k=None):
    """Piecewise-polynomial coefficients in s = (th - th_i) / h from node values y and
    theta-derivatives: cubic Hermite [n-1, 4] from the slopes m; with the second
    derivatives k, quintic Hermite [n-1, 6] (value, slope and curvature matched at both
    nodes).  D = y_i+1 - y_i, a = h m, b = h^2 k:
      cubic   c = [y_i, a_i, 3D - 2a_i - a_i+1, a_i + a_i+1 - 2D]
      quintic c = [y_i, a_i, b_i/2, 10D - 6a_i - 4a_i+1 - (3b_i - b_i+1)/2,
                   -15D + 8a_i + 7a_i+1 + (3b_i - 2b_i+1)/2, 6D - 3(a_i + a_i+1) - (b_i - b_i+1)/2]"""
    y = np.asarray(y, dtype=float)
    a = h * np.asarray(m, dtype=float)
    d = y[1:] - y[:-1]
    a0, a1 = a[:-1], a[1:]
    if k is None:
        return np.stack([y[:-1], a0, 3 * d - 2 * a0 - a1, a0 + a1 - 2 * d], axis=-1)
    b = h * h * np.asarray(k, dtype=float)
    b0, b1 = b[:-1], b[1:]
    return np.stack([y[:-1], a0, b0 / 2, 10 * d - 6 * a0 - 4 * a1 - (3 * b0 - b1) / 2,
                     -15 * d + 8 * a0 + 7 * a1 + (3 * b0 - 2 * b1) / 2, 6 * d - 3 * (a0 + a1) - (b0 - b1) / 2],
                    axis=-1)


def tabulate_electrode(hd: SynthHandles, th, T_K, order=1):
    """An Electrode from closed-form handles: v2 node tables (the handle values at the
    (T, theta) nodes), and with ``order`` 3 / 5 the v3 cubic / quintic Hermite
    coefficients of each row, with the Arrhenius factor of ``hd.energies()`` divided out
    of the rows."""
    th = np.asarray(th, dtype=float)
    T_K = np.atleast_1d(np.asarray(T_K, dtype=float))
    h = 1.0 / (th.size - 1)
    cubic = order > 1
    ea = hd.energies() if cubic else {}
    tabs, coefs = {}, {}
    for name in EL_TABLES:
        vals, cs = [], []
        for T in T_K:
            y, m, k = hd.rows(name, th, T)
            if not cubic and name in ("k0", "Rf"):    # v2: the handle's values, factor included
                f = hd._arr(hd.Ea_k0 if name == "k0" else -hd.Ea_rf, T)
                y = y * f
            vals.append(y)
            cs.append(hermite_coefs(y, m, h, k if order == 5 else None))
        tabs[name] = np.array(vals)
        coefs[name] = np.array(cs)
    u1, m1, k1 = hd.rows("Uocp1", th, hd.Tref)
    coefs["Uocp1"] = hermite_coefs(u1, m1, h, k1 if order == 5 else None)
    return Electrode(theta0=hd.th0, theta100=hd.th100, soc0=np.full(T_K.size, hd.th0),
                     soc100=np.full(T_K.size, hd.th100), Uocp=tabs["Uocp"], Uocp1=u1, dUocp=tabs["dUocp"],
                     k0=tabs["k0"], Rf=tabs["Rf"], Cdleff=tabs["Cdleff"],
                     poly=coefs if cubic else None, Ea=ea or None)


# ---------------------------------------------------------------------------------------
# The exporter's algorithm for arbitrary handles (matlab/mpcekf_tabulate_electrode.m and
# mpcekf_export_rom.m run the same steps on a MATLAB ROM's cellData.function; this mirror
# lets the steps be tested here against the closed-form synthetic handles as black boxes)
# ---------------------------------------------------------------------------------------
FD_STEP = 1e-4   # finite-difference step of the exporter's theta-derivatives


def fd_derivs(f, th, e=FD_STEP):
    """(f, f', f'') of a scalar function at the nodes th by 5-point stencils of step e:
    central inside [2e, 1 - 2e], shifted one-sided (forward / backward, 4th / 3rd order)
    at the ends so no stencil point leaves [0, 1] (a handle need not extrapolate)."""
    th = np.asarray(th, dtype=float)
    y = np.array([f(t) for t in th])
    d1, d2 = np.empty_like(y), np.empty_like(y)
    for i, t in enumerate(th):
        if 2 * e <= t <= 1 - 2 * e:
            fm2, fm1, fp1, fp2 = f(t - 2 * e), f(t - e), f(t + e), f(t + 2 * e)
            d1[i] = (-fp2 + 8 * fp1 - 8 * fm1 + fm2) / (12 * e)
            d2[i] = (-fp2 + 16 * fp1 - 30 * y[i] + 16 * fm1 - fm2) / (12 * e * e)
        else:
            s = 1.0 if t < 2 * e else -1.0        # stencil into the interval
            g = [f(t + s * k * e) for k in range(1, 5)]
            d1[i] = s * (-25 * y[i] + 48 * g[0] - 36 * g[1] + 16 * g[2] - 3 * g[3]) / (12 * e)
            d2[i] = (35 * y[i] - 104 * g[0] + 114 * g[1] - 56 * g[2] + 11 * g[3]) / (12 * e * e)
    return y, d1, d2


def detect_arrhenius(f, T_K, Tref, R, th=None, tol=1e-10):
    """Ea (J/mol) when f(th, T) = f(th, Tref) exp(Ea/R (1/Tref - 1/T)) on the sample (the
    ratio is theta-independent and log-linear in 1/T, both to tol), else 0.0."""
    th = np.linspace(0.03, 0.97, 13) if th is None else th
    Ts = [T for T in np.atleast_1d(T_K) if abs(T - Tref) > 1e-6]
    if not Ts:
        return 0.0
    base = np.array([f(t, Tref) for t in th])
    if not np.all(np.isfinite(base)) or np.any(base == 0):
        return 0.0
    eas = []
    for T in Ts:
        r = np.array([f(t, T) for t in th]) / base
        if not np.all(np.isfinite(r)) or np.any(r <= 0) or np.ptp(r) > tol * abs(r[0]):
            return 0.0
        eas.append(R * math.log(float(np.mean(r))) / (1.0 / Tref - 1.0 / T))
    ea = float(np.mean(eas))
    if ea == 0.0 or max(abs(x - ea) for x in eas) > 1e-8 * abs(ea):
        return 0.0
    return ea


NODE_FNS = EL_TABLES + ("Uocp1",)


def discover_nodes(ws, lo=-1e-12, hi=1.0 + 1e-12):
    """The theta breakpoints a lookup-table handle carries (matlab/mpcekf_handle_nodes.m: MATLAB's
    functions(h).workspace{1}, recursing into captured handles): the union of every captured
    strictly ascending finite numeric vector of >= 3 values inside [0, 1].  None for a
    closed-form handle.  A captured vector that is not a breakpoint set only refines the
    segments, which keeps a piecewise polynomial exact."""
    found = []

    def walk(v, depth=0):
        if depth > 8:
            return
        if isinstance(v, dict):
            for x in v.values():
                walk(x, depth + 1)
        elif callable(v) and hasattr(v, "workspace"):
            walk(v.workspace(), depth + 1)
        elif isinstance(v, (list, tuple, np.ndarray)):
            a = np.asarray(v)
            if a.dtype.kind in "fiu" and a.ndim >= 1 and a.squeeze().ndim == 1:
                a = a.astype(float).ravel()
                if (a.size >= 3 and np.all(np.isfinite(a)) and np.all(np.diff(a) > 0)
                        and a[0] >= lo and a[-1] <= hi):
                    found.append(a)
    walk(ws)
    if not found:
        return None
    return np.unique(np.clip(np.concatenate(found), 0.0, 1.0))


_T4 = np.array([0.0, 1.0 / 3.0, 2.0 / 3.0, 1.0])
_V4INV = np.linalg.inv(np.vander(_T4, 4, increasing=True))


def fit_segments(f, x):
    """ABI v4 coefficients [m-1, 4] of a piecewise cubic with breakpoints x from handle calls
    alone: per segment the cubic through f at x_k + h (0, 1/3, 2/3, 1), in s = theta - x_k.
    Exact (to rounding) for any handle that is a polynomial of degree <= 3 on every segment
    -- interp1 'linear', pchip, spline, makima.  A segment whose quadratic and cubic terms are
    rounding noise is stored as interp1's (y_k, (y_k+1 - y_k) / h, 0, 0)."""
    x = np.asarray(x, dtype=float)
    c = np.zeros((x.size - 1, 4))
    for k in range(x.size - 1):
        a, b = float(x[k]), float(x[k + 1])
        h = b - a
        ys = np.array([f(a), f(a + h / 3.0), f(a + 2.0 * h / 3.0), f(b)])
        q = _V4INV @ ys
        scale = max(float(np.max(np.abs(ys))), 1e-300)
        if abs(q[2]) <= 64 * EPS * scale and abs(q[3]) <= 64 * EPS * scale:
            c[k] = (ys[0], (ys[3] - ys[0]) / h, 0.0, 0.0)
        else:
            c[k] = (q[0], q[1] / h, q[2] / (h * h), q[3] / (h * h * h))
    return c


def tabulate_nodes(fh, T_K, Tref=298.15, R=8.3144621, ea=None):
    """The ABI v4 node tables {name: (x, coef)} of every function of handle object fh whose
    workspace carries breakpoints (discover_nodes); ea {name: J/mol} as detect_arrhenius
    found them (the rows of such a function are taken at Tref)."""
    if not hasattr(fh, "workspace"):
        return {}
    T_K = np.atleast_1d(np.asarray(T_K, dtype=float))
    ea = ea or {}
    fns = {"Uocp": fh.Uocp, "dUocp": fh.dUocp, "k0": fh.k0, "Rf": fh.Rf, "Cdleff": fh.Cdleff}
    out = {}
    for name in NODE_FNS:
        x = discover_nodes(fh.workspace(name))
        if x is None or x.size < 2:
            continue
        if name == "Uocp1":
            out[name] = (x, fit_segments(lambda t: fh.Uocp(t), x))
            continue
        f = fns[name]
        rows = []
        for T in T_K:
            Tr = Tref if ea.get(name, 0.0) != 0.0 else T
            rows.append(fit_segments(lambda t, Tr=Tr: f(t, Tr), x))
        out[name] = (x, np.array(rows))
    return out


def tabulate_handles(fh, ntheta, T_K, Tref=298.15, R=8.3144621, order=5, nodes=False):
    """An ABI v3 Electrode from a handle object with the cellData.function interface
    (Uocp(th, T), Uocp(th), dUocp, k0, Rf, Cdleff, soc(z, T), theta0(), theta100()),
    using only handle calls -- the exporter's algorithm (matlab/mpcekf_tabulate_electrode.m):

    * per function, an Arrhenius factor when detect_arrhenius finds one; its rows are then
      the function at Tref at every table temperature (identical rows: the library reads
      one), else the function at each table temperature;
    * theta-derivatives by fd_derivs; Hermite cubics (order 3) or quintics (order 5) of
      every row (hermite_coefs); the v2 node tables alongside (the handle's values);
    * nodes=True (ABI v4): also the node tables of the functions whose handle workspace
      carries breakpoints (tabulate_nodes); the library then looks those up on their own
      nodes and the uniform-grid polynomials of the others."""
    th = np.linspace(0.0, 1.0, int(ntheta))
    T_K = np.atleast_1d(np.asarray(T_K, dtype=float))
    h = 1.0 / (th.size - 1)
    fns = {"Uocp": fh.Uocp, "dUocp": fh.dUocp, "k0": fh.k0, "Rf": fh.Rf, "Cdleff": fh.Cdleff}
    ea, tabs, coefs = {}, {}, {}
    for name, f in fns.items():
        e = detect_arrhenius(f, T_K, Tref, R)
        if e != 0.0:
            ea[name] = e
        vals, cs = [], []
        for T in T_K:
            Tr = Tref if e != 0.0 else T
            y, d1, d2 = fd_derivs(lambda t, Tr=Tr: f(t, Tr), th)
            cs.append(hermite_coefs(y, d1, h, d2 if order == 5 else None))
            vals.append(np.array([f(t, T) for t in th]))     # v2 node table: the handle itself
        tabs[name] = np.array(vals)
        coefs[name] = np.array(cs)
    y, d1, d2 = fd_derivs(lambda t: fh.Uocp(t), th)
    coefs["Uocp1"] = hermite_coefs(y, d1, h, d2 if order == 5 else None)
    nd = tabulate_nodes(fh, T_K, Tref, R, ea) if nodes else {}
    return Electrode(theta0=float(fh.theta0()), theta100=float(fh.theta100()),
                     soc0=np.array([fh.soc(0.0, T) for T in T_K]), soc100=np.array([fh.soc(1.0, T) for T in T_K]),
                     Uocp=tabs["Uocp"], Uocp1=y, dUocp=tabs["dUocp"], k0=tabs["k0"], Rf=tabs["Rf"],
                     Cdleff=tabs["Cdleff"], poly=coefs, Ea=ea or None, nodes=nd or None)


def budget_ok(err):
    return all(err[k] <= TABLE_BUDGET[k] for k in TABLE_BUDGET)


class TableBudgetError(ValueError):
    """The exported lookups miss TABLE_BUDGET (matlab/mpcekf_build_tables.m refuses such a ROM)."""

    def __init__(self, msg, err):
        super().__init__(msg)
        self.err = err


def export_electrodes(handles, T_K, Tref=298.15, R=8.3144621, T_eval=None, order=5, nodes=True,
                      ntheta=None, thlim=None, strict=True):
    """The exporter's whole table step for both electrodes (matlab/mpcekf_build_tables.m, the
    helper mpcekf_export_rom and the OB_step drop-in share): node tables where a handle's
    workspace carries breakpoints and they meet the budget, the uniform-grid polynomials for
    the rest, with ntheta doubled from 257 to 4097 until every function meets TABLE_BUDGET at
    T_eval (default: the table temperatures and their midpoints) over each electrode's
    operating theta range.  Returns ({"neg": Electrode, "pos": ...}, ntheta, errors).  When the
    budget is missed at 4097: TableBudgetError (strict) or the last tables with their errors."""
    T_K = np.atleast_1d(np.asarray(T_K, dtype=float))
    sizes = [int(ntheta)] if ntheta else [257, 513, 1025, 2049, 4097]
    errs = {}
    els = {}
    for nth in sizes:
        ok = True
        for side, fh in handles.items():
            e = tabulate_handles(fh, nth, T_K, Tref, R, order, nodes=nodes)
            lo, hi = thlim[side] if thlim else (0.0, 1.0)
            err = table_errors(fh, e, T_K, Tref, R, lo, hi, T_eval=T_eval)
            if e.nodes:   # a node table that misses the budget falls back to the uniform grid
                bad = [k for k in list(e.nodes) if not _fn_ok(fh, e, k, T_K, Tref, R, lo, hi, T_eval)]
                for k in bad:
                    del e.nodes[k]
                if bad:
                    err = table_errors(fh, e, T_K, Tref, R, lo, hi, T_eval=T_eval)
                e.nodes = e.nodes or None
            els[side], errs[side] = e, err
            ok = ok and budget_ok(err)
        if ok:
            return els, nth, errs
    if strict:
        raise TableBudgetError(f"the electrode tables miss the error budget at {sizes[-1]} theta points: {errs}",
                               errs)
    return els, sizes[-1], errs


_FN_BUDGET = {"Uocp": "Uocp", "Uocp1": "Uocp", "dUocp": "dUocp_rel", "k0": "k0_rel", "Rf": "Rf_rel",
              "Cdleff": "Cdleff_rel"}


def _fn_ok(fh, e, name, T_K, Tref, R, lo, hi, T_eval):
    """One function's node table against its TABLE_BUDGET entry (table_errors restricted)."""
    err = table_errors(fh, e, T_K, Tref, R, lo, hi, T_eval=T_eval, only=name)
    return err[_FN_BUDGET[name]] <= TABLE_BUDGET[_FN_BUDGET[name]]


# error budget of the exported tables (matlab/mpcekf_check_tables.m): north_star's 1e-6
# relative is 80 nV on phise (~0.08 V), into which Uocp_n enters directly
# (EKFmatsHandler.m:96); the tables are held to a tenth of it
TABLE_BUDGET = {"Uocp": 8e-9, "dUocp_rel": 1e-7, "k0_rel": 1e-9, "Rf_rel": 1e-9, "Cdleff_rel": 1e-3, "soc_lin": 1e-12}


def table_errors(fh, e: Electrode, T_K, Tref=298.15, R=8.3144621, theta_lo=0.0, theta_hi=1.0, n=997,
                 T_eval=None, only=None):
    """Largest differences of the v3 / v4 lookups from the handles (matlab/mpcekf_check_tables.m):
    at n theta points inside [theta_lo, theta_hi] and at T_eval, by default every table
    temperature and the midpoints between them (a caller that knows the temperatures the
    simulation runs at -- the OB_step drop-in's Tc -- passes those).  only: one function
    (NODE_FNS name; "Uocp1" is the one-argument Uocp)."""
    T_K = np.atleast_1d(np.asarray(T_K, dtype=float))
    cf = CellFunctions(e, T_K, R, Tref)
    xs = np.linspace(theta_lo, theta_hi, n)
    Ts = np.sort(np.concatenate([T_K, (T_K[1:] + T_K[:-1]) / 2])) if T_eval is None else np.atleast_1d(T_eval)
    err = {k: 0.0 for k in TABLE_BUDGET}
    names = ("dUocp", "k0", "Rf", "Cdleff") if only is None else tuple(k for k in (only,) if k in EL_TABLES[1:])
    for T in Ts:
        for x in xs:
            if only in (None, "Uocp"):
                err["Uocp"] = max(err["Uocp"], abs(cf.Uocp(x, T) - fh.Uocp(x, T)))
            for nm in names:
                ref = getattr(fh, nm)(x, T)
                err[nm + "_rel"] = max(err[nm + "_rel"], abs(getattr(cf, nm)(x, T) - ref) / max(abs(ref), 1e-300))
            if only is None:
                s0, s1 = fh.soc(0.0, T), fh.soc(1.0, T)
                err["soc_lin"] = max(err["soc_lin"], abs(fh.soc(x, T) - (s0 + x * (s1 - s0))))
    if only in (None, "Uocp1"):
        for x in xs:
            err["Uocp"] = max(err["Uocp"], abs(cf.Uocp(x) - fh.Uocp(x)))
    return err


def synth_handles(R=8.3144621, Tref=298.15):
    """(neg, pos) closed-form handles of the synthetic NMC30-like cell."""
    neg = SynthHandles(theta0=0.01, theta100=0.80, u=_u_neg, du=_du_neg, d2u=_d2u_neg, d3u=_d3u_neg,
                       dudt=lambda x: -1.0e-4 * np.exp(-5 * x), ddudt=lambda x: 5.0e-4 * np.exp(-5 * x),
                       d2dudt=lambda x: -2.5e-3 * np.exp(-5 * x), d3dudt=lambda x: 1.25e-2 * np.exp(-5 * x), k0ref=2.0, Ea_k0=3.0e4, Rf=2.0e-3,
                       Ea_rf=1.0e4, wDL=5.0, Cdl=150.0, nDL=0.95, R=R, Tref=Tref)
    pos = SynthHandles(theta0=0.93, theta100=0.40, u=_u_pos, du=_du_pos, d2u=_d2u_pos, d3u=_d3u_pos,
                       dudt=lambda x: -0.5e-4 * (1 - x), ddudt=lambda x: 0.5e-4 + 0.0 * x,
                       d2dudt=lambda x: 0.0 * x, d3dudt=lambda x: 0.0 * x, k0ref=4.0, Ea_k0=4.0e4, Rf=3.0e-3, Ea_rf=1.0e4, wDL=5.0,
                       Cdl=120.0, nDL=0.93, R=R, Tref=Tref)
    return neg, pos


def make_synth_rom(T_degC=(15.0, 25.0, 35.0), SOC_pct=tuple(range(0, 101, 5)), Ts=1.0,
                   ntab=None, tab_T_degC=None, lookup="linear") -> ROM:
    """Deterministic synthetic NMC30-like xRA ROM.

    Every number is fixed here; nothing random.  Local models differ smoothly with
    temperature (Arrhenius) and SOC so the bilinear blends of OB_step.m:281-285 and
    iterEKF.m:312-313 exercise real interpolation.  The electrode handles
    (:func:`synth_handles`, attached as ``rom.handles``) are tabulated on ``tab_T_degC``
    x ``ntab`` theta points (include/mpcekf.h mpcekf_electrode):

    * ``lookup="linear"`` (ABI v2, the default of the round-1..4 fixtures): node values,
      linear in theta and T; ``ntab`` default 201;
    * ``lookup="cubic"`` / ``"quintic"`` (ABI v3): Hermite cubics / quintics in theta
      from the handles' values and theta-derivatives, k0 / Rf with their exact Arrhenius
      factor; ``ntab`` default 1025 / 513 (the quintic follows the handles
      to the ulp level on the outputs, the cubic to ~1e-10).
    """
    order = {"linear": 1, "cubic": 3, "quintic": 5}.get(lookup)
    if order is None:
        raise ValueError(f"lookup {lookup!r}: 'linear', 'cubic' or 'quintic'")
    if tab_T_degC is None:   # v3: rows past the operating range (an affine OCP is exact between rows, not beyond)
        tab_T_degC = (5.0, 25.0, 45.0) if lookup == "linear" else (-10.0, 25.0, 60.0)
    if ntab is None:   # DESIGN.md §3 (tools/handle_gap.py): the quintic at 513 points follows the handles to ulps
        ntab = {"linear": 201, "cubic": 1025, "quintic": 513}[lookup]
    T_degC = np.asarray(T_degC, dtype=float)
    SOC_pct = np.asarray(SOC_pct, dtype=float)
    R = 8.3144621
    F = 96485.3365
    Q = 29.86
    Tref = 298.15
    n = 5
    nT, nZ, nz = len(T_degC), len(SOC_pct), len(_OUTPUTS)

    th = np.linspace(0.0, 1.0, ntab)
    T_K = np.asarray(tab_T_degC, dtype=float) + 273.15
    hn, hp = synth_handles(R, Tref)
    if lookup == "linear":   # the round-1..4 tables, bit for bit (their fixtures are keyed by this ROM's hash)
        neg = _synth_electrode(T_K, th, Tref, R, theta0=0.01, theta100=0.80, u=_u_neg,
                               dudt=lambda x: -1.0e-4 * np.exp(-5 * x), k0ref=2.0, Ea_k0=3.0e4, Rf=2.0e-3,
                               Ea_rf=1.0e4, wDL=5.0, Cdl=150.0, nDL=0.95)
        pos = _synth_electrode(T_K, th, Tref, R, theta0=0.93, theta100=0.40, u=_u_pos,
                               dudt=lambda x: -0.5e-4 * (1 - x), k0ref=4.0, Ea_k0=4.0e4, Rf=3.0e-3,
                               Ea_rf=1.0e4, wDL=5.0, Cdl=120.0, nDL=0.93)
    else:
        neg = tabulate_electrode(hn, th, T_K, order=order)
        pos = tabulate_electrode(hp, th, T_K, order=order)
    res0n = -Ts * (neg.theta100 - neg.theta0) / (3600 * Q)
    res0p = -Ts * (pos.theta100 - pos.theta0) / (3600 * Q)

    A = np.zeros((nT, nZ, n + 1))
    C = np.zeros((nT, nZ, nz, n + 1))
    D = np.zeros((nT, nZ, nz))
    for t in range(nT):
        TK = T_degC[t] + 273.15
        f_res = math.exp(2.0e4 / R * (1.0 / TK - 1.0 / Tref))   # resistive gains
        f_tau = math.exp(1.5e4 / R * (1.0 / TK - 1.0 / Tref))   # slower when cold
        for z in range(nZ):
            zz = SOC_pct[z] / 100.0
            f_soc = 1.0 + 0.3 * (zz - 0.5) ** 2
            tau = _TAU_REF * f_tau * (1.0 + 0.2 * (zz - 0.5) ** 2) * np.array([1.0, 1.02, 1.05, 1.1, 1.2])
            a = np.exp(-Ts / tau)
            A[t, z, :n] = a
            A[t, z, n] = 1.0
            for r, (nm, _loc, d, g, r0) in enumerate(_OUTPUTS):
                if nm in _FLUX:
                    scale = 1.0 + 0.1 * (zz - 0.5)
                elif "Thetass" in nm or "Thetae" in nm:
                    scale = f_tau
                else:
                    scale = f_res * f_soc
                C[t, z, r, :n] = np.asarray(g, dtype=float) * scale * (1.0 - a)
                D[t, z, r] = d * scale
                C[t, z, r, n] = res0n if r0 == "n" else (res0p if r0 == "p" else 0.0)
    rom = ROM(T_degC=T_degC, SOC_pct=SOC_pct, Ts=float(Ts), A=A, C=C, D=D,
              names=[o[0] for o in _OUTPUTS], xloc=np.array([o[1] for o in _OUTPUTS]),
              F=F, R=R, Q=Q, Rc=8.0e-4, Tref=Tref, tab_T_K=T_K, neg=neg, pos=pos,
              meta={"kind": "synthetic-NMC30-like", "version": 2 if lookup == "linear" else 3,
                    "lookup": lookup})
    rom.handles = {"neg": hn, "pos": hp}
    rom.validate()
    return rom


# ---------------------------------------------------------------------------------------
# A second synthetic handle family: lookup-table handles (round 6)
# ---------------------------------------------------------------------------------------
# A ROM from the Plett-Trimboli toolchain (README.md:61) commonly carries its OCP as measured
# data interpolated on the data's own, non-uniform breakpoints, e.g.
#   Uocp = @(x,T) interp1(xU, U0, x) + (T - Tref) * interp1(xS, dS, x)
# which is neither smooth nor of the closed forms SynthHandles has.  TabHandles is such a cell:
# the same NMC30-like curves, but sampled ("measured") at breakpoints clustered at the theta
# ends and interpolated linearly (interp1) or by pchip; an entropic dU/dT table on its own,
# coarser breakpoints; dUocp from tabulated derivative data; k0 with a tabulated theta factor
# and a two-term (not pure Arrhenius) temperature dependence.  workspace(name) mirrors
# MATLAB's functions(h).workspace{1}, where the exporter finds the breakpoints.

def pchip_slopes(x, y):
    """MATLAB pchip's node slopes (Fritsch-Butland: the weighted harmonic mean of the
    neighbouring secants inside, zero at a sign change; the shape-preserving three-point
    formula at the ends)."""
    x, y = np.asarray(x, float), np.asarray(y, float)
    h = np.diff(x)
    dl = np.diff(y) / h
    n = x.size
    d = np.zeros(n)
    for k in range(1, n - 1):
        if dl[k - 1] * dl[k] > 0:
            w1, w2 = 2 * h[k] + h[k - 1], h[k] + 2 * h[k - 1]
            d[k] = (w1 + w2) / (w1 / dl[k - 1] + w2 / dl[k])

    def end(h0, h1, d0, d1):
        s = ((2 * h0 + h1) * d0 - h0 * d1) / (h0 + h1)
        if np.sign(s) != np.sign(d0):
            s = 0.0
        elif np.sign(d0) != np.sign(d1) and abs(s) > abs(3 * d0):
            s = 3 * d0
        return s
    d[0] = end(h[0], h[1], dl[0], dl[1])
    d[-1] = end(h[-1], h[-2], dl[-1], dl[-2])
    return d


class _Table:
    """y(x) on breakpoints x: interp1 'linear' (clamped to the end values outside [x0, x_end],
    as the library's theta is clamped to [0, 1]) or 'pchip' (ppval: local Horner, end pieces
    extended)."""

    def __init__(self, x, y, kind="linear"):
        self.x, self.y, self.kind = np.asarray(x, float), np.asarray(y, float), kind
        if kind == "pchip":
            x, y = self.x, self.y
            h = np.diff(x)
            dl = np.diff(y) / h
            d = pchip_slopes(x, y)
            self.c = np.stack([y[:-1], d[:-1], (3 * dl - 2 * d[:-1] - d[1:]) / h,
                               (d[:-1] - 2 * dl + d[1:]) / (h * h)], axis=-1)

    def __call__(self, t):
        t = float(t)
        if self.kind == "linear":
            return float(np.interp(t, self.x, self.y))
        k = int(np.clip(np.searchsorted(self.x, t, side="right") - 1, 0, self.x.size - 2))
        s = t - self.x[k]
        c = self.c[k]
        return float(c[0] + s * (c[1] + s * (c[2] + s * c[3])))

    def deriv_data(self):
        """Derivative data at the breakpoints, as a toolchain tabulates dU/dx next to U."""
        return np.gradient(self.y, self.x, edge_order=2) if self.kind == "linear" else pchip_slopes(self.x, self.y)


def clustered_nodes(m_mid=72, m_end=12, edge=0.05, seed=0):
    """Breakpoints as measured OCP data has them: m_end points over each of [0, edge] and
    [1 - edge, 1], m_mid over the middle, interior ones jittered by up to 20 % of the local
    spacing (deterministic)."""
    rng = np.random.Generator(np.random.PCG64(0x7AB + seed))
    x = np.unique(np.concatenate([np.linspace(0.0, edge, m_end + 1), np.linspace(edge, 1 - edge, m_mid + 1),
                                  np.linspace(1 - edge, 1.0, m_end + 1)]))
    h = np.diff(x)
    j = rng.uniform(-0.2, 0.2, x.size - 2) * np.minimum(h[:-1], h[1:])
    x[1:-1] += j
    return x


class TabHandles:
    """Lookup-table ``cellData.function.{neg,pos}`` handles (see the section comment)."""

    def __init__(self, *, theta0, theta100, u, dudt, kth, Ea_k0, Rf, Ea_rf, wDL, Cdl, nDL, R, Tref, kind="linear",
                 seed=0):
        self.th0, self.th100, self.R, self.Tref, self.kind = theta0, theta100, R, Tref, kind
        xU = clustered_nodes(seed=seed)
        xS = np.linspace(0.0, 1.0, 31)
        xS[1:-1] += np.random.Generator(np.random.PCG64(0x5A + seed)).uniform(-0.005, 0.005, 29)
        xk = np.array([0.0, 0.1, 0.22, 0.35, 0.5, 0.63, 0.78, 0.9, 1.0])
        self.U0 = _Table(xU, u(xU), kind)                    # measured OCP at Tref
        self.dS = _Table(xS, dudt(xS), "linear")             # entropic coefficient table
        self.dU0 = _Table(xU, self.U0.deriv_data(), "linear")
        self.ddS = _Table(xS, self.dS.deriv_data(), "linear")
        self.kt = _Table(xk, kth(xk), "linear")
        self.Ea1, self.Ea2 = Ea_k0                           # two-term kinetics
        self.Rf0, self.Ea_rf = Rf, Ea_rf
        self.wDL, self.Cdl, self.nDL = wDL, Cdl, nDL

    def workspace(self, name):
        """What MATLAB's functions(h).workspace{1} would show for the handle ``name``."""
        U = {"xU": self.U0.x, "U0": self.U0.y, "xS": self.dS.x, "dS": self.dS.y, "Tref": self.Tref}
        if name == "Uocp":
            return U
        if name == "Uocp1":
            return {"xU": self.U0.x, "U0": self.U0.y}
        if name == "dUocp":
            return {"xU": self.dU0.x, "dU0": self.dU0.y, "xS": self.ddS.x, "ddS": self.ddS.y, "Tref": self.Tref}
        if name == "k0":
            return {"xk": self.kt.x, "kk": self.kt.y, "Ea1": self.Ea1, "Ea2": self.Ea2, "R": self.R}
        if name == "Rf":
            return {"Rf0": self.Rf0, "Ea": self.Ea_rf, "R": self.R}
        return {"Cdl": self.Cdl, "wDL": self.wDL, "nDL": self.nDL}

    def theta0(self):
        return self.th0

    def theta100(self):
        return self.th100

    def soc(self, z, T):
        return self.th0 + z * (self.th100 - self.th0)

    def Uocp(self, th, T=None):
        if T is None:
            return self.U0(th)
        return self.U0(th) + (T - self.Tref) * self.dS(th)

    def dUocp(self, th, T):
        return self.dU0(th) + (T - self.Tref) * self.ddS(th)

    def _arr(self, Ea, T):
        return math.exp(Ea / self.R * (1.0 / self.Tref - 1.0 / T))

    def k0(self, th, T):
        return self.kt(th) * (0.6 * self._arr(self.Ea1, T) + 0.4 * self._arr(self.Ea2, T))

    def Rf(self, th, T):
        return float(self.Rf0 * self._arr(-self.Ea_rf, T) * (0.8 + 0.4 * th))

    def Cdleff(self, th, T):
        cdl = self.Cdl * (1.0 + 2e-3 * (T - self.Tref))
        return float((cdl ** (2 - self.nDL)) * (self.wDL ** (self.nDL - 1)))


def tab_handles(kind="linear", R=8.3144621, Tref=298.15):
    """(neg, pos) lookup-table handles of the synthetic NMC30-like cell (TabHandles)."""
    neg = TabHandles(theta0=0.01, theta100=0.80, u=_u_neg, dudt=lambda x: -1.0e-4 * np.exp(-5 * x),
                     kth=lambda x: 2.0 * (0.9 + 0.4 * x * (1 - x)), Ea_k0=(3.0e4, 5.0e4), Rf=2.0e-3, Ea_rf=1.0e4,
                     wDL=5.0, Cdl=150.0, nDL=0.95, R=R, Tref=Tref, kind=kind, seed=0)
    pos = TabHandles(theta0=0.93, theta100=0.40, u=_u_pos, dudt=lambda x: -0.5e-4 * (1 - x),
                     kth=lambda x: 4.0 * (0.9 + 0.4 * x * (1 - x)), Ea_k0=(4.0e4, 2.0e4), Rf=3.0e-3, Ea_rf=1.0e4,
                     wDL=5.0, Cdl=120.0, nDL=0.93, R=R, Tref=Tref, kind=kind, seed=1)
    return neg, pos


def operating_theta(h, pad=0.04):
    """The electrode's theta range over 0-100 % SOC widened by pad (mpcekf_export_rom's lim)."""
    a, b = h.soc(0.0, h.Tref), h.soc(1.0, h.Tref)
    return max(0.0, min(a, b) - pad), min(1.0, max(a, b) + pad)


def make_tab_rom(kind="linear", tab_T_degC=(-10.0, 25.0, 60.0), nodes=True, T_eval_degC=None, ntheta=None,
                 strict=True) -> ROM:
    """The synthetic cell's models (make_synth_rom) with the lookup-table handles of
    tab_handles(kind), exported by the exporter's algorithm (export_electrodes) from handle
    calls alone: ABI v4 node tables for the interp1 / pchip functions (nodes=True), the
    uniform-grid quintics otherwise.  T_eval_degC: the temperatures the budget is checked at
    (default the table temperatures and midpoints).  rom.handles = the handles (the numpy
    oracle's handle mode); rom.meta["tab_error"] = the exporter's errors."""
    base = make_synth_rom(lookup="quintic", ntab=257)
    hn, hp = tab_handles(kind, base.R, base.Tref)
    T_K = np.asarray(tab_T_degC, dtype=float) + 273.15
    T_eval = None if T_eval_degC is None else np.asarray(T_eval_degC, dtype=float) + 273.15
    els, nth, errs = export_electrodes({"neg": hn, "pos": hp}, T_K, base.Tref, base.R, T_eval=T_eval, nodes=nodes,
                                       ntheta=ntheta, thlim={"neg": operating_theta(hn), "pos": operating_theta(hp)},
                                       strict=strict)
    rom = ROM(T_degC=base.T_degC, SOC_pct=base.SOC_pct, Ts=base.Ts, A=base.A, C=base.C, D=base.D, names=base.names,
              xloc=base.xloc, F=base.F, R=base.R, Q=base.Q, Rc=base.Rc, Tref=base.Tref, tab_T_K=T_K,
              neg=els["neg"], pos=els["pos"],
              meta={"kind": f"synthetic-NMC30-like, {kind} lookup-table handles", "version": 4 if nodes else 3,
                    "lookup": "nodes" if nodes else "quintic", "ntheta": nth, "tab_error": errs})
    rom.handles = {"neg": hn, "pos": hp}
    rom.validate()
    return rom
