/*
 * oracle/mpcekf_oracle.c -- scalar C restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  It is the checker for the HIP kernels and the
 * "port" CPU baseline of bench.py; nothing in the product links or calls it.
 *
 * PARITY UNPINNED: the reference (MATLAB, Rodrigops27/MPC-EKF4FastCharge) cannot
 * run in this image and ships no fixtures; see oracle/oracle_np.py's header and
 * DESIGN.md "Oracle".  This file restates, per cell:
 *   OB_step.m:188-357 (simStep)          -> orc_plant_step
 *   iterEKF.m:30-602  ('OB' branches)     -> orc_ekf_step and helpers
 *   EKFmatsHandler.m:26-114               -> orc_mats_handler
 *   predMat.m:11-53                       -> orc_predmat
 *   constraintsMPC.m:15-112               -> orc_constraints
 *   hildreth.m:17-46                      -> orc_hildreth
 *   iterMPC.m:17-95                       -> orc_mpc_step
 *   initKF.m:30-136, initMPC.m:29-74      -> orc_init_cell
 *   runMPC.m:72-112 (loop order)          -> orc_run
 * Conventions (shared with oracle_np.py and the kernels): sequential dot
 * products from +0.0, no FMA contraction (build with -ffp-contract=off),
 * MATLAB max/min ignore NaN, Cholesky for E\X, LU for (-E)\x.
 * Differences from oracle_np.py by design: covariances are stored packed
 * (upper triangle, 15 doubles) and the SVD symmetrisation of iterEKF.m:143-145
 * is evaluated with a cyclic Jacobi eigensolver of the symmetric part.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Defined asinh, the same spelling as dasinh in mpcekf_kernels.hip (the overpotential
 * of OB_step.m:333-334, iterEKF.m:400-401, EKFmatsHandler.m:88-89).  glibc's asinh is not
 * correctly rounded, and neither is the GPU's, so both sides evaluate log(u) + c with
 * u = 2^k m, m in (sqrt(2)/2, sqrt(2)], and the minimax series in s = f / (2 + f),
 * f = m - 1 (fdlibm's published Lg1..Lg7).  Only +, -, *, /, sqrt and fma. */
static const double DM_LN2_HI = 6.93147180369123816490e-01, DM_LN2_LO = 1.90821492927058770002e-10;
static const double DM_LN2 = 6.93147180559945286227e-01;
static const double DM_LG1 = 6.666666666666735130e-01, DM_LG2 = 3.999999999940941908e-01,
                    DM_LG3 = 2.857142874366239149e-01, DM_LG4 = 2.222219843214978396e-01,
                    DM_LG5 = 1.818357216161805012e-01, DM_LG6 = 1.531383769920937332e-01,
                    DM_LG7 = 1.479819860511658591e-01;

static double dm_log_core(double u, double c) { /* log(u) + c, u >= 1 finite */
  uint64_t b;
  memcpy(&b, &u, 8);
  int k = (int)(b >> 52) - 1023;
  uint64_t mb = (b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;
  double m;
  memcpy(&m, &mb, 8);
  if (m > 1.4142135623730951) { m = 0.5 * m; k = k + 1; }
  double f = m - 1.0;
  double s = f / (2.0 + f);
  double z = s * s;
  double w = z * z;
  double t1 = w * (DM_LG2 + w * (DM_LG4 + w * DM_LG6));
  double t2 = z * (DM_LG1 + w * (DM_LG3 + w * (DM_LG5 + w * DM_LG7)));
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  double dk = (double)k;
  return dk * DM_LN2_HI - ((hfsq - (s * (hfsq + R) + (dk * DM_LN2_LO + c))) - f);
}

double orc_asinh(double x) {
  double a = fabs(x);
  if (!(a < INFINITY)) return x + x;
  if (a < 0x1p-28) return x;
  double t;
  if (a > 0x1p28) {
    t = dm_log_core(a, 0.0) + DM_LN2;
  } else if (a > 2.0) {
    t = dm_log_core(2.0 * a + 1.0 / (sqrt(fma(a, a, 1.0)) + a), 0.0);
  } else { /* log1p(a + a^2 / (1 + sqrt(1 + a^2))) */
    double a2 = a * a;
    double xx = a + a2 / (1.0 + sqrt(1.0 + a2));
    double u = 1.0 + xx;
    double c = (xx - (u - 1.0)) / u;
    t = dm_log_core(u, c);
  }
  return x < 0 ? -t : t;
}
#define dasinh orc_asinh

#define NX 5
#define NPK 15
#define NPMAX 20
#define NCMAX 10
#define NCONMAX (4 * NCMAX + 3 * NPMAX)

enum { TF_negIfdl, TF_posIfdl, TF_negIf, TF_posIf, TF_negIdl, TF_posIdl, TF_negPhis, TF_posPhis,
       TF_negPhise, TF_posPhise, TF_negThetass, TF_posThetass, TF_negPhie, TF_sepPhie,
       TF_posPhie, TF_negThetae, TF_sepThetae, TF_posThetae };

enum { ST_ERROR = 1, ST_LOCKOUT = 2, ST_THETAE_NEG = 4 };

/* cellData.function.{neg,pos} tabulated on (rom.TK x uniform theta over [0,1]) */
typedef struct {
  double theta0, theta100;                       /* zero-argument calls (OB_step.m:207-210) */
  const double *soc0, *soc100;                   /* [ntemp] */
  const double *Uocp, *dUocp, *k0, *Rf, *Cdleff; /* [ntemp][ntheta] */
  const double *Uocp1;                           /* [ntheta] one-argument Uocp (EKFmatsHandler.m:96) */
  /* ABI v3 (include/mpcekf.h): theta polynomials [ntemp][ntheta-1][6] ([ntheta-1][6] for
   * Uocp1), all NULL for linear tables; Arrhenius energies of Uocp, dUocp, k0, Rf, Cdleff */
  const double *Uocp_p, *dUocp_p, *k0_p, *Rf_p, *Cdleff_p, *Uocp1_p;
  double Ea[5];
  int tconst; /* bit f: every row of function f's polynomials is the same (row 0 blended with itself) */
  /* ABI v4 (include/mpcekf.h): function f (Uocp, dUocp, k0, Rf, Cdleff, Uocp1) on its own
   * theta nodes when nnode[f] >= 2: node[f] [m], node_p[f] [ntemp][m-1][6] ([m-1][6]) */
  int nnode[6];
  const double *node[6], *node_p[6];
} orc_electrode;

typedef struct {
  int nT, nZ, n, nz;
  const double *T_degC, *SOC_pct;
  double Ts;
  const double *A;   /* [nT][nZ][n+1]     */
  const double *C;   /* [nT][nZ][nz][n+1] */
  const double *D;   /* [nT][nZ][nz]      */
  const int32_t *tf; /* [nz] TF_* codes   */
  const double *xloc;
  double F, R, Q, Rc, Tref;
  int ntheta, ntemp;
  const double *TK; /* [ntemp] table temperatures (K, ascending) */
  orc_electrode neg, pos;
} orc_rom;
enum { EF_U = 0, EF_DU, EF_K0, EF_RF, EF_CDL };
#define NPOLY 6 /* coefficients per theta interval of the v3 tables (a cubic's upper two are 0) */

typedef struct {
  int Np, Nc;
  double ref, u_max, Crate, du_min, du_max, v_max, phise_min, z_max, z_tol;
  int use_cur, use_v, use_eta;
  int maxHild;
  double hild_tol;
  double SigmaV, SigmaW;
  double SigmaX0[NX + 1]; /* diagonal of SigmaX0 (runMPC.m:17) */
  int max_warn;           /* iterEKF.m:55: lockout when warnCount > max_warn */
  int method;             /* 0 = 'OB' output blend (runMPC.m), 1 = 'MB' model blend (initKF.m:44-49) */
} orc_cfg;

/* resolved output indices (iterEKF.m:610-735) */
typedef struct {
  int Ifdl0, Ifdl3, If0, If3, Thetass0, Thetass3, Phise0, Thetae1, ThetaeE, PhieE, negPhise2;
  int nNegTh, negTh[32], nPosTh, posTh[32], nNegPhise, negPhise[32], nPosPhise, posPhise[32];
  int nPhie, Phie[32], PhieLoc0[32], nThetae, Thetae[32], nPosPhis, posPhis[32];
} orc_ind;

typedef struct {
  /* plant (OB_step cellState) */
  double *bigX; /* [NM][NX+1] */
  double SOCnAvg, SOCpAvg, SOC0n, SOC0p, Tc;
  /* ekf */
  double *xhat; /* [NM][NX] */
  double *S;    /* [NM][NPK] */
  double x0, S0, priorI, SOC0;
  /* 'MB': one shared model state (x0 above is its integrator, xhat(end)) and one full
   * (NX+1)x(NX+1) covariance (initKF.m:100-101) */
  double xmb[NX], Smb[(NX + 1) * (NX + 1)];
  int warn, status;
  /* mpc */
  double uk_1, uk;
  double lam[NCONMAX];
} orc_cell;

static const int PK[NX][NX] = {{0, 1, 2, 3, 4}, {1, 5, 6, 7, 8}, {2, 6, 9, 10, 11},
                               {3, 7, 10, 12, 13}, {4, 8, 11, 13, 14}};

/* boundzk's quadratic forms row' * Sigma * row (iterEKF.m:191-197, diagonal only) in the
 * symmetric form the k_bounds kernel spells: T = Sigma with doubled off-diagonals,
 * u_k = T_kk r_k + sum_{l>k} T_kl r_l, q = sum_k r_k u_k, every step an explicit fma()
 * (correctly rounded here and on the GPU, so both sides agree bit for bit). */
static void qform_prep(const double S[NPK], double T[NPK]) {
  for (int k = 0; k < NX; ++k)
    for (int l = k; l < NX; ++l) T[PK[k][l]] = k == l ? S[PK[k][l]] : 2 * S[PK[k][l]];
}
static double qform(const double T[NPK], const double r[NX]) {
  double q = 0.0;
  for (int k = 0; k < NX; ++k) {
    double u = T[PK[k][k]] * r[k];
    for (int l = k + 1; l < NX; ++l) u = fma(T[PK[k][l]], r[l], u);
    q = k == 0 ? r[0] * u : fma(r[k], u, q);
  }
  return q;
}

/* ----------------------------------------------------------------------- */
/* cellData.function.* (tabulated, see rom.py)                              */
/* ----------------------------------------------------------------------- */
static double tab_interp(const double *tab, int n, double x) {
  if (x != x) return NAN;
  double xc = fmin(fmax(x, 0.0), 1.0);
  double t = xc * (double)(n - 1);
  int i = (int)floor(t);
  if (i > n - 2) i = n - 2;
  double f = t - (double)i;
  return tab[i] + f * (tab[i + 1] - tab[i]);
}
/* the table temperature bracket of T: clamp to the grid ends, j = last index with
 * TK[j] <= T (at most ntemp - 2), g = (T - TK[j]) / (TK[j+1] - TK[j]) */
static void tidx(const orc_rom *r, double T, int *j, double *g) {
  *j = 0;
  *g = 0.0;
  if (r->ntemp == 1) return;
  double Tc = fmin(fmax(T, r->TK[0]), r->TK[r->ntemp - 1]);
  int k = 0;
  while (k < r->ntemp - 2 && Tc >= r->TK[k + 1]) ++k;
  *j = k;
  *g = (Tc - r->TK[k]) / (r->TK[k + 1] - r->TK[k]);
}
/* ABI v3 row: the polynomial of theta's interval, Horner with explicit fma over 6
 * coefficients in s = t - i (mpcekf_kernels.hip tabp; rom.py interp_poly without fma) */
static double tab_poly(const double *c, int n, double x) {
  if (x != x) return NAN;
  double xc = fmin(fmax(x, 0.0), 1.0);
  double t = xc * (double)(n - 1);
  int i = (int)floor(t);
  if (i > n - 2) i = n - 2;
  double s = t - (double)i;
  const double *p = c + (size_t)i * NPOLY;
  double v = p[5];
  v = fma(s, v, p[4]);
  v = fma(s, v, p[3]);
  v = fma(s, v, p[2]);
  v = fma(s, v, p[1]);
  return fma(s, v, p[0]);
}
/* ABI v4 row (include/mpcekf.h node / node_p): theta clamped to [0, 1], its segment
 * k = #{j in 1..m-2 : x_j <= theta} (found by bisection here; the kernels read it from a
 * uniform bucket map built to give this k), then Horner with explicit fma over 6
 * coefficients in s = theta - x_k (rom.py interp_nodes without fma) */
static double node_poly(const double *x, int m, const double *c, double th) {
  if (th != th) return NAN;
  const double xc = fmin(fmax(th, 0.0), 1.0);
  int lo = 0, hi = m - 2; /* the largest k in [0, m-2] with k == 0 or x[k] <= xc */
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (x[mid] <= xc) lo = mid;
    else hi = mid - 1;
  }
  const double s = xc - x[lo];
  const double *p = c + (size_t)lo * NPOLY;
  double v = p[5];
  v = fma(s, v, p[4]);
  v = fma(s, v, p[3]);
  v = fma(s, v, p[2]);
  v = fma(s, v, p[1]);
  return fma(s, v, p[0]);
}
/* Defined exp (the v3 Arrhenius factor; rom.py dexp, mpcekf_kernels.hip dexp): fdlibm's
 * reduction x = k ln2 + r (k = floor(x / ln2 + 1/2)) and its rational form for exp(r);
 * +, -, *, /, floor and ldexp only, each exact or correctly rounded on both sides. */
static const double EXP_P1 = 1.66666666666666019037e-01, EXP_P2 = -2.77777777770155933842e-03,
                    EXP_P3 = 6.61375632143793436117e-05, EXP_P4 = -1.65339022054652515390e-06,
                    EXP_P5 = 4.13813679705723846039e-08, EXP_INVLN2 = 1.44269504088896338700e+00;
double orc_exp(double x) {
  if (x != x) return x;
  if (x > 709.782712893384) return INFINITY;
  if (x < -745.1332191019412) return 0.0;
  double k = floor(x * EXP_INVLN2 + 0.5);
  double hi = x - k * DM_LN2_HI;
  double lo = k * DM_LN2_LO;
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (EXP_P1 + t * (EXP_P2 + t * (EXP_P3 + t * (EXP_P4 + t * EXP_P5))));
  double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  return ldexp(y, (int)k);
}
/* One handle lookup (include/mpcekf.h): the rows j, j+1 of the T bracket at
 * theta (linear in the node values, or the v3 polynomials), a + g (b - a), then the
 * Arrhenius factor exp(Ea/R (1/Tref - 1/T)) when Ea != 0 (T unclamped). */
static double tab2(const orc_rom *r, const orc_electrode *e, int f, const double *t, const double *tp, double th,
                   double T) {
  const double Ea = e->Ea[f];
  const int one = (e->tconst >> f) & 1;
  int j;
  double g;
  tidx(r, T, &j, &g);
  const size_t rp = (size_t)(r->ntheta - 1) * NPOLY;
  double a;
  if (e->nnode[f] >= 2) { /* v4: the function's own nodes, rows blended as v3's */
    const int m = e->nnode[f];
    const size_t np = (size_t)(m - 1) * NPOLY;
    if (one) j = 0;
    a = node_poly(e->node[f], m, e->node_p[f] + j * np, th);
    const double b = (one || r->ntemp == 1) ? a : node_poly(e->node[f], m, e->node_p[f] + (j + 1) * np, th);
    a = a + g * (b - a);
  } else if (tp) {
    /* v3: rows j and j + 1 blended; a T-invariant function (all rows equal, `one`) or a
     * single-temperature table blends row 0 with itself, a + g (a - a) (the library's one
     * lookup path, mpcekf_kernels.hip ETab::f) */
    if (one) j = 0;
    a = tab_poly(tp + j * rp, r->ntheta, th);
    const double b = (one || r->ntemp == 1) ? a : tab_poly(tp + (j + 1) * rp, r->ntheta, th);
    a = a + g * (b - a);
  } else {
    a = tab_interp(t + (size_t)j * r->ntheta, r->ntheta, th);
    if (r->ntemp > 1) {
      double b = tab_interp(t + (size_t)(j + 1) * r->ntheta, r->ntheta, th);
      a = a + g * (b - a);
    }
  }
  if (Ea != 0.0) a = a * orc_exp((Ea / r->R) * (1.0 / r->Tref - 1.0 / T));
  return a;
}
static double tab1T(const orc_rom *r, const double *t, double T) {
  int j;
  double g;
  tidx(r, T, &j, &g);
  if (r->ntemp == 1) return t[0];
  return t[j] + g * (t[j + 1] - t[j]);
}
/* soc(z,T) (iterEKF.m:282-283; EKFmatsHandler.m:57-58; OB_step.m:64-65) */
static double fsoc(const orc_rom *r, const orc_electrode *e, double z, double T) {
  double s0 = tab1T(r, e->soc0, T), s1 = tab1T(r, e->soc100, T);
  return s0 + z * (s1 - s0);
}
static double fUocp(const orc_rom *r, const orc_electrode *e, double th, double T) {
  return tab2(r, e, EF_U, e->Uocp, e->Uocp_p, th, T);
}
static double fUocp1(const orc_rom *r, const orc_electrode *e, double th) {
  if (e->nnode[5] >= 2) return node_poly(e->node[5], e->nnode[5], e->node_p[5], th);
  return e->Uocp1_p ? tab_poly(e->Uocp1_p, r->ntheta, th) : tab_interp(e->Uocp1, r->ntheta, th);
}
static double fdUocp(const orc_rom *r, const orc_electrode *e, double th, double T) {
  return tab2(r, e, EF_DU, e->dUocp, e->dUocp_p, th, T);
}
static double fk0(const orc_rom *r, const orc_electrode *e, double th, double T) {
  return tab2(r, e, EF_K0, e->k0, e->k0_p, th, T);
}
static double fRf(const orc_rom *r, const orc_electrode *e, double th, double T) {
  return tab2(r, e, EF_RF, e->Rf, e->Rf_p, th, T);
}
static double fCdl(const orc_rom *r, const orc_electrode *e, double th, double T) {
  return tab2(r, e, EF_CDL, e->Cdleff, e->Cdleff_p, th, T);
}
static double msqrt(double x) { return x >= 0 ? sqrt(x) : NAN; }

/* ----------------------------------------------------------------------- */
/* index resolution                                                          */
/* ----------------------------------------------------------------------- */
int orc_resolve(const orc_rom *r, orc_ind *ix) {
  memset(ix, 0, sizeof(*ix));
  int Ifdl0 = -1, Ifdl3 = -1, If0 = -1, If3 = -1, Th0 = -1, Th3 = -1, Ph0 = -1, nph = 0;
  int ifdl[64], nifdl = 0, iff[64], niff = 0, ths[64], nths = 0, phs[64], nphs = 0;
  /* concatenation order [neg; pos] and [neg; sep; pos] as in iterEKF.m:656-670 */
  for (int pass = 0; pass < 2; ++pass)
    for (int i = 0; i < r->nz; ++i) {
      int c = r->tf[i];
      if (c == (pass ? TF_posIfdl : TF_negIfdl)) ifdl[nifdl++] = i;
      if (c == (pass ? TF_posIf : TF_negIf)) iff[niff++] = i;
      if (c == (pass ? TF_posThetass : TF_negThetass)) ths[nths++] = i;
      if (c == (pass ? TF_posPhise : TF_negPhise)) phs[nphs++] = i;
    }
  for (int k = 0; k < nifdl; ++k) {
    if (r->xloc[ifdl[k]] == 0) Ifdl0 = ifdl[k];
    if (r->xloc[ifdl[k]] == 3) Ifdl3 = ifdl[k];
  }
  for (int k = 0; k < niff; ++k) {
    if (r->xloc[iff[k]] == 0) If0 = iff[k];
    if (r->xloc[iff[k]] == 3) If3 = iff[k];
  }
  for (int k = 0; k < nths; ++k) {
    if (r->xloc[ths[k]] == 0) Th0 = ths[k];
    if (r->xloc[ths[k]] == 3) Th3 = ths[k];
  }
  for (int k = 0; k < nphs; ++k)
    if (r->xloc[phs[k]] == 0) Ph0 = phs[k];
  if (Ifdl0 < 0 || Ifdl3 < 0 || If0 < 0 || If3 < 0 || Th0 < 0 || Th3 < 0 || Ph0 < 0) return -1;
  ix->Ifdl0 = Ifdl0; ix->Ifdl3 = Ifdl3; ix->If0 = If0; ix->If3 = If3;
  ix->Thetass0 = Th0; ix->Thetass3 = Th3; ix->Phise0 = Ph0;
  for (int pass = 0; pass < 3; ++pass)
    for (int i = 0; i < r->nz; ++i) {
      int c = r->tf[i];
      int want_e = pass == 0 ? TF_negPhie : pass == 1 ? TF_sepPhie : TF_posPhie;
      int want_t = pass == 0 ? TF_negThetae : pass == 1 ? TF_sepThetae : TF_posThetae;
      if (c == want_e) { ix->Phie[ix->nPhie] = i; ix->PhieLoc0[ix->nPhie] = r->xloc[i] == 0; ix->nPhie++; }
      if (c == want_t) ix->Thetae[ix->nThetae++] = i;
    }
  if (ix->nPhie > 0 && ix->PhieLoc0[0]) { /* iterEKF.m:728-731 */
    for (int k = 1; k < ix->nPhie; ++k) { ix->Phie[k - 1] = ix->Phie[k]; ix->PhieLoc0[k - 1] = ix->PhieLoc0[k]; }
    ix->nPhie--;
  }
  if (ix->nPhie == 0 || ix->nThetae == 0) return -2;
  ix->PhieE = ix->Phie[ix->nPhie - 1];
  ix->Thetae1 = ix->Thetae[0];
  ix->ThetaeE = ix->Thetae[ix->nThetae - 1];
  for (int i = 0; i < r->nz; ++i) {
    int c = r->tf[i];
    if (c == TF_negThetass) ix->negTh[ix->nNegTh++] = i;
    if (c == TF_posThetass) ix->posTh[ix->nPosTh++] = i;
    if (c == TF_negPhise) ix->negPhise[ix->nNegPhise++] = i;
    if (c == TF_posPhise) ix->posPhise[ix->nPosPhise++] = i;
    if (c == TF_posPhis) ix->posPhis[ix->nPosPhis++] = i;
  }
  if (ix->nNegPhise < 2) return -3;
  ix->negPhise2 = ix->negPhise[1];
  (void)nph;
  return 0;
}

/* ----------------------------------------------------------------------- */
/* small dense linear algebra (defined order)                               */
/* ----------------------------------------------------------------------- */
/* E\B via Cholesky, B is n x m column-major in b[c*n + i]; returns 0 on success */
static int chol_solve(int n, const double *E /* n x n row-major */, int m, const double *B, double *X) {
  double R[NCMAX * NCMAX];
  for (int j = 0; j < n; ++j) {
    double s = E[j * n + j];
    for (int k = 0; k < j; ++k) s = s - R[k * n + j] * R[k * n + j];
    if (!(s > 0)) return -1;
    R[j * n + j] = sqrt(s);
    for (int i = j + 1; i < n; ++i) {
      double t = E[j * n + i];
      for (int k = 0; k < j; ++k) t = t - R[k * n + j] * R[k * n + i];
      R[j * n + i] = t / R[j * n + j];
    }
  }
  for (int c = 0; c < m; ++c) {
    double y[NCMAX];
    for (int i = 0; i < n; ++i) {
      double t = B[c * n + i];
      for (int k = 0; k < i; ++k) t = t - R[k * n + i] * y[k];
      y[i] = t / R[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double t = y[i];
      for (int k = i + 1; k < n; ++k) t = t - R[i * n + k] * X[c * n + k];
      X[c * n + i] = t / R[i * n + i];
    }
  }
  return 0;
}

static void lu_solve(int n, const double *Ain, const double *b, double *x) {
  double A[NCMAX * NCMAX], y[NCMAX];
  memcpy(A, Ain, sizeof(double) * n * n);
  memcpy(y, b, sizeof(double) * n);
  for (int k = 0; k < n; ++k) {
    int p = k;
    for (int i = k + 1; i < n; ++i)
      if (fabs(A[i * n + k]) > fabs(A[p * n + k])) p = i;
    if (p != k) {
      for (int j = 0; j < n; ++j) { double t = A[k * n + j]; A[k * n + j] = A[p * n + j]; A[p * n + j] = t; }
      double t = y[k]; y[k] = y[p]; y[p] = t;
    }
    for (int i = k + 1; i < n; ++i) {
      double l = A[i * n + k] / A[k * n + k];
      A[i * n + k] = l;
      for (int j = k + 1; j < n; ++j) A[i * n + j] = A[i * n + j] - l * A[k * n + j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < i; ++k) y[i] = y[i] - A[i * n + k] * y[k];
  for (int i = n - 1; i >= 0; --i) {
    double t = y[i];
    for (int k = i + 1; k < n; ++k) t = t - A[i * n + k] * x[k];
    x[i] = t / A[i * n + i];
  }
}

static void mldivide_spd(int n, const double *E, int m, const double *B, double *X) {
  if (chol_solve(n, E, m, B, X) == 0) return;
  for (int c = 0; c < m; ++c) lu_solve(n, E, B + c * n, X + c * n);
}

/* Cyclic Jacobi eigensolver, symmetric n x n (row-major, overwritten). */
void orc_jacobi(int n, double *a, double *V, double *w) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0, dg = 0.0;
    for (int p = 0; p < n; ++p) {
      dg = dg + a[p * n + p] * a[p * n + p];
      for (int q = p + 1; q < n; ++q) off = off + a[p * n + q] * a[p * n + q];
    }
    if (!(off > 1e-36 * dg)) break;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        double apq = a[p * n + q];
        if (apq == 0.0) continue;
        double theta = (a[q * n + q] - a[p * n + p]) / (2.0 * apq);
        double t;
        if (fabs(theta) > 1e150) t = 0.5 / theta;
        else {
          t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
          if (theta < 0) t = -t;
        }
        double c = 1.0 / sqrt(t * t + 1.0), s = t * c, tau = s / (1.0 + c);
        a[p * n + p] = a[p * n + p] - t * apq;
        a[q * n + q] = a[q * n + q] + t * apq;
        a[p * n + q] = 0.0;
        a[q * n + p] = 0.0;
        for (int r = 0; r < n; ++r) {
          if (r == p || r == q) continue;
          double g = a[r * n + p], h = a[r * n + q];
          double gn = g - s * (h + g * tau), hn = h + s * (g - h * tau);
          a[r * n + p] = gn; a[p * n + r] = gn;
          a[r * n + q] = hn; a[q * n + r] = hn;
        }
        for (int r = 0; r < n; ++r) {
          double g = V[r * n + p], h = V[r * n + q];
          V[r * n + p] = g - s * (h + g * tau);
          V[r * n + q] = h + s * (g - h * tau);
        }
      }
  }
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

/* sigma_min of the symmetric PSD Nc x Nc matrix (iterMPC.m:41-43) */
double orc_sigma_min(int n, const double *G) {
  double a[NCMAX * NCMAX], V[NCMAX * NCMAX], w[NCMAX];
  memcpy(a, G, sizeof(double) * n * n);
  orc_jacobi(n, a, V, w);
  double m = fabs(w[0]);
  for (int i = 1; i < n; ++i)
    if (fabs(w[i]) < m) m = fabs(w[i]);
  return m;
}

/* iterEKF.m:141-151 on one packed covariance.
 * P = Sigma - (L*St)*L' ; S_new = ((P + P') + HH + HH')/4 with HH = V|D|V',
 * V,D from Jacobi of (P+P')/2 ; then Q-bump x2. */
/* Positive definiteness of a symmetric NX x NX matrix by LDL' pivots (no square
 * roots): every pivot d_j > 0.  The kernels evaluate the identical sequence. */
int orc_is_pd(const double *a /*full, symmetric*/) {
  double l[NX][NX], d[NX];
  for (int j = 0; j < NX; ++j) {
    double s = a[j * NX + j];
    for (int k = 0; k < j; ++k) s = fma(-(l[j][k] * l[j][k]), d[k], s);
    if (!(s > 0)) return 0;
    d[j] = s;
    double inv = 1.0 / s;
    for (int i = j + 1; i < NX; ++i) {
      double t = a[i * NX + j];
      for (int k = 0; k < j; ++k) t = fma(-(l[i][k] * l[j][k]), d[k], t);
      l[i][j] = t * inv;
    }
  }
  return 1;
}

void orc_meas_cov(double *S /*packed*/, const double *L, double St, int bump) {
  double P[NX][NX], a[NX * NX], V[NX * NX], w[NX];
  double LS[NX];
  for (int r = 0; r < NX; ++r) LS[r] = L[r] * St;
  for (int r = 0; r < NX; ++r)
    for (int c = 0; c < NX; ++c) P[r][c] = fma(-LS[r], L[c], S[PK[r][c]]);
  for (int r = 0; r < NX; ++r)
    for (int c = 0; c < NX; ++c) a[r * NX + c] = (P[r][c] + P[c][r]) * 0.5;
  /* HH = VV*SS*VV' of svd (iterEKF.m:145-146) is the polar factor of SigmaX; for the
   * symmetric part a it is V|Lambda|V' (Jacobi).  When a is positive definite that
   * is a itself: take it directly (no reconstruction rounding) and skip the
   * eigen-decomposition. */
  double HH[NX][NX];
  if (orc_is_pd(a)) {
    for (int r = 0; r < NX; ++r)
      for (int c = 0; c < NX; ++c) HH[r][c] = a[r * NX + c];
  } else {
    orc_jacobi(NX, a, V, w);
    for (int r = 0; r < NX; ++r)
      for (int c = 0; c < NX; ++c) {
        double acc = 0.0;
        for (int k = 0; k < NX; ++k) acc = acc + (V[r * NX + k] * fabs(w[k])) * V[c * NX + k];
        HH[r][c] = acc;
      }
  }
  for (int r = 0; r < NX; ++r)
    for (int c = r; c < NX; ++c) {
      double v = (((P[r][c] + P[c][r]) + HH[r][c]) + HH[c][r]) / 4.0;
      if (bump) v = v * 2.0;
      S[PK[r][c]] = v;
    }
}

/* ----------------------------------------------------------------------- */
/* predMat.m with A = diag(a), B = ones: Phi (Np x 7), G (Np x Nc)           */
/* ----------------------------------------------------------------------- */
void orc_predmat(const double *a /*6*/, const double *C /*6*/, double D, int Np, int Nc, double *Phi,
                 double *G) {
  const int nx = NX + 1, na = NX + 2;
  double Abar[7][7], X[7], Ap[7][7], H[NPMAX], Cbar[7];
  memset(Abar, 0, sizeof(Abar));
  for (int i = 0; i < nx; ++i) { Abar[i][i] = a[i]; Abar[i][nx] = 1.0; }
  Abar[nx][nx] = 1.0;
  for (int i = 0; i < nx; ++i) Cbar[i] = C[i];
  Cbar[nx] = D;
  for (int i = 0; i < na; ++i) X[i] = 0.0;
  X[nx] = 1.0;
  for (int k = 0; k < Np; ++k) {
    double acc = 0.0;
    for (int j = 0; j < na; ++j) acc = acc + Cbar[j] * X[j];
    H[k] = acc;
    double Xn[7];
    for (int i = 0; i < na; ++i) {
      double s = 0.0;
      for (int j = 0; j < na; ++j) s = s + Abar[i][j] * X[j];
      Xn[i] = s;
    }
    memcpy(X, Xn, sizeof(X));
  }
  for (int i = 0; i < na; ++i)
    for (int j = 0; j < na; ++j) Ap[i][j] = i == j ? 1.0 : 0.0;
  for (int i = 0; i < Np; ++i) {
    double An[7][7];
    for (int r = 0; r < na; ++r)
      for (int c = 0; c < na; ++c) {
        double s = 0.0;
        for (int k = 0; k < na; ++k) s = s + Abar[r][k] * Ap[k][c];
        An[r][c] = s;
      }
    memcpy(Ap, An, sizeof(Ap));
    for (int c = 0; c < na; ++c) {
      double s = 0.0;
      for (int k = 0; k < na; ++k) s = s + Cbar[k] * Ap[k][c];
      Phi[i * na + c] = s;
    }
    for (int j = 0; j < Nc; ++j) G[i * Nc + j] = j <= i ? H[i - j] : 0.0;
  }
}

/* ----------------------------------------------------------------------- */
/* hildreth.m                                                               */
/* ----------------------------------------------------------------------- */
/* v = X*lambda, X(:,j) = E\M(j,:)' stored row j of X[] (sums from +0, ascending j) */
static void hild_v(int Nc, int nC, const double *X, const double *lam, double *v) {
  for (int k = 0; k < Nc; ++k) {
    double a = 0.0;
    for (int j = 0; j < nC; ++j) a = fma(X[j * Nc + k], lam[j], a);
    v[k] = a;
  }
}

/* t_i = K_i + M(i,:)*v of the rank form.  Nc <= 2 (the lane-per-cell kernels): fma in
 * ascending k.  Nc > 2 (the 8-lane-group kernels, lane k holding v_k and v_{k+8}):
 * a_0 = fma(M_i0, v_0, K_i), a_k = M_ik*v_k for 0 < k < min(Nc, 8), +0 for Nc <= k < 8;
 * b_k = fma(M_i,k+8, v_k+8, a_k) when k + 8 < Nc, else a_k; summed as the pairwise tree
 * ((b0+b1)+(b2+b3)) + ((b4+b5)+(b6+b7)) (the 3-level lane butterfly).  For Nc <= 8 this is
 * round 2's 16-slot tree up to the sign of a zero t (its extra slots only added +0), which
 * cannot reach lambda: min(t (1/H_ii), lambda_i) is then +-0 or lambda_i, and lambda_i - m and
 * the step's effect on v are the same for either sign (hild_step). */
static double hild_row_t(int Nc, const double *Mi, const double *v, double Ki) {
  if (Nc <= 2) {
    double t = Ki;
    for (int k = 0; k < Nc; ++k) t = fma(Mi[k], v[k], t);
    return t;
  }
  double b[8];
  for (int k = 0; k < 8; ++k) b[k] = k == 0 ? fma(Mi[0], v[0], Ki) : (k < Nc ? Mi[k] * v[k] : 0.0);
  for (int k = 8; k < Nc; ++k) b[k - 8] = fma(Mi[k], v[k], b[k - 8]);
  for (int w = 1; w < 8; w *= 2)
    for (int k = 0; k < 8; k += 2 * w) b[k] = b[k] + b[k + w];
  return b[0];
}

/* hildreth.m:35-36's update, lambda_i <- max(0, w) with w = -(K_i + H(i,:)*lambda - H_ii lambda_i)
 * / H_ii = lambda_i - t_i / H_ii (t_i = K_i + H(i,:)*lambda): the defined spelling (round 6)
 * takes the step, not the new value, first -- d = max(-lambda_i, -t_i / H_ii) = -min(q, lambda_i)
 * with q = t_i * (1/H_ii) (1/H_ii once per solve and row), lambda_i <- lambda_i - min(q,
 * lambda_i).  So the per-row chain is t -> q -> min -> (v += X(:,i) d), the new lambda_i
 * beside it, and an inactive row (q >= lambda_i) lands on +0 exactly.  fmin(NaN, l) = l: a NaN
 * q leaves lambda_i = 0, as max(0, NaN) = 0 does.  The step d = -min(q, lambda_i) is what v is
 * updated with and what the stop test (hildreth.m:39) measures.  Outside the reciprocal's
 * normal range (|H_ii| not 0 and outside [2^-1020, 2^1020]) or with a non-finite lambda_i (an
 * inf lambda_i with H_ii = 0 is NaN in MATLAB's H_ii * lambda_i term): the division form,
 * w = fma(H_ii, lambda_i, -t_i) / H_ii, new = max(w, 0), d = new - lambda_i.  H_ii = +-0 (the
 * SOC block's first row, predMat G(1,1) = 0): 1/H_ii = +-inf, and q = t * (+-inf) gives x / +-0's
 * inf / NaN by IEEE, as the division does.  Returns d; *nl = the new lambda_i. */
static int hild_rok(double h) {
  const double a = fabs(h);
  return h == 0.0 || (a >= 0x1p-1020 && a <= 0x1p1020);
}
static double hild_step(double t, double h, double rinv, double l, double *nl) {
  if (hild_rok(h) && isfinite(l)) {
    const double m = fmin(t * rinv, l);
    *nl = l - m;
    return -m;
  }
  const double w = fma(h, l, -t) / h;
  *nl = w > 0 ? w : 0.0;
  return *nl - l;
}

int orc_hildreth(int Nc, int nC, const double *E, const double *F, const double *M /*nC x Nc*/,
                 const double *gam, double *lam /*in: warm start, out*/, int maxIter, double tol,
                 double *DU) {
  static const int HMAX = NCONMAX;
  double *H = (double *)malloc(sizeof(double) * HMAX * HMAX);
  double Mt[NCMAX * NCONMAX], X[NCMAX * NCONMAX], y[NCMAX], K[NCONMAX];
  for (int i = 0; i < nC; ++i)
    for (int k = 0; k < Nc; ++k) Mt[i * Nc + k] = M[i * Nc + k]; /* column i of M' */
  mldivide_spd(Nc, E, nC, Mt, X);                                /* X(:,i) = E\M(i,:)' */
  for (int i = 0; i < nC; ++i)
    for (int j = 0; j < nC; ++j) {
      double s = 0.0;
      for (int k = 0; k < Nc; ++k) s = s + M[i * Nc + k] * X[j * Nc + k];
      H[i * HMAX + j] = s;
    }
  mldivide_spd(Nc, E, 1, F, y);
  for (int i = 0; i < nC; ++i) {
    double s = 0.0;
    for (int k = 0; k < Nc; ++k) s = s + M[i * Nc + k] * y[k];
    K[i] = s + gam[i];
  }
  /* H = M*X has rank Nc: H(i,:)*lambda = M(i,:)*v with v = X*lambda (an Nc-vector).
   * Defined evaluation (the kernels evaluate the same sequence):
   *  - finite X and M: v recomputed from lambda at the start of every sweep (fma
   *    accumulation from +0 in ascending j), t_i = K_i + M(i,:)*v as hild_row_t,
   *    the step d and new lambda_i by hild_step (lambda_i - t_i / H_ii clamped at 0), and
   *    after row i v += X(:,i)*(new - old lambda(i)) by fma; when that change is not
   *    finite (a zero-diagonal row going to or from +inf) v is recomputed from lambda
   *    instead, which reproduces the dense form's inf/NaN propagation in kind.
   *  - otherwise the dense H(i,:)*lambda as 4 interleaved partial sums (terms j = q
   *    mod 4 from +0) combined as (p0+p1)+(p2+p3).
   * MATLAB's own BLAS order for H(i,:)*lambda is unpinned; the math is hildreth.m:35. */
  int finite = 1;
  for (int i = 0; i < nC * Nc; ++i) finite = finite && isfinite(X[i]) && isfinite(M[i]);
  int it = 0;
  for (it = 1; it <= maxIter; ++it) {
    int conv = 1;
    double v[NCMAX];
    if (finite) hild_v(Nc, nC, X, lam, v);
    for (int i = 0; i < nC; ++i) {
      double nl, d, hii = H[i * HMAX + i];
      if (finite) {
        double t = hild_row_t(Nc, M + i * Nc, v, K[i]);
        d = hild_step(t, hii, 1.0 / hii, lam[i], &nl);
      } else {
        double p[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = 0; j < nC; ++j) p[j & 3] = p[j & 3] + H[i * HMAX + j] * lam[j];
        double s = (p[0] + p[1]) + (p[2] + p[3]);
        const double w = -((K[i] + s) - hii * lam[i]) / hii;
        nl = w > 0 ? w : 0.0;
        d = nl - lam[i];
      }
      if (!(fabs(d) < tol)) conv = 0;
      lam[i] = nl;
      if (finite) {
        if (isfinite(d))
          for (int k = 0; k < Nc; ++k) v[k] = fma(X[i * Nc + k], d, v[k]);
        else
          hild_v(Nc, nC, X, lam, v);
      }
    }
    if (conv) break;
  }
  if (it > maxIter) it = maxIter;
  double rhs[NCMAX], mE[NCMAX * NCMAX];
  for (int k = 0; k < Nc; ++k) {
    double s = 0.0;
    for (int i = 0; i < nC; ++i) s = s + M[i * Nc + k] * lam[i];
    rhs[k] = F[k] + s;
  }
  for (int i = 0; i < Nc * Nc; ++i) mE[i] = -E[i];
  lu_solve(Nc, mE, rhs, DU);
  free(H);
  return it;
}

/* ----------------------------------------------------------------------- */
/* per-cell model                                                           */
/* ----------------------------------------------------------------------- */
typedef struct {
  const orc_rom *r;
  const orc_cfg *c;
  orc_ind ix;
  int NM;
  double Tpts[64], Zpts[64]; /* sorted set-points: K and fraction */
  double smin;               /* sigma_min(Gsoc'Gsoc) is evaluated per step below */
} orc_ctx;

static void two_nearest(const double *pts, int n, double x, int *i1, int *i2) {
  int b1 = -1, b2 = -1;
  double d1 = 0, d2 = 0;
  for (int i = 0; i < n; ++i) {
    double d = fabs(x - pts[i]);
    /* stable ascending sort, NaN last */
    int better1 = b1 < 0 || (d < d1) || (d1 != d1 && d == d);
    if (better1) { b2 = b1; d2 = d1; b1 = i; d1 = d; continue; }
    int better2 = b2 < 0 || (d < d2) || (d2 != d2 && d == d);
    if (better2) { b2 = i; d2 = d; }
  }
  *i1 = b1;
  *i2 = b2 < 0 ? b1 : b2;
}

typedef struct {
  double g[4];
  int m[4]; /* model index t*nZ + z */
} orc_xind;

static void get_xind(const orc_ctx *X, double Tk, double SOC, orc_xind *xi) {
  const orc_rom *r = X->r;
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (r->nZ > 1) {
    int a, b;
    two_nearest(X->Zpts, r->nZ, SOC, &a, &b);
    iZu = a; iZl = b;
    if (X->Zpts[iZu] < X->Zpts[iZl]) { iZu = b; iZl = a; }
  }
  if (r->nT > 1) {
    int a, b;
    two_nearest(X->Tpts, r->nT, Tk, &a, &b);
    iTu = a; iTl = b;
    if (X->Tpts[iTu] < X->Tpts[iTl]) { iTu = b; iTl = a; }
  }
  double aZ = 0.0, aT = 0.0;
  if (r->nZ > 1) aZ = (SOC - X->Zpts[iZl]) / (X->Zpts[iZu] - X->Zpts[iZl]);
  if (r->nT > 1) aT = (Tk - X->Tpts[iTl]) / (X->Tpts[iTu] - X->Tpts[iTl]);
  xi->g[0] = (1 - aT) * (1 - aZ);
  xi->g[1] = (1 - aT) * aZ;
  xi->g[2] = aT * (1 - aZ);
  xi->g[3] = aT * aZ;
  xi->m[0] = iTl * r->nZ + iZl;
  xi->m[1] = iTl * r->nZ + iZu;
  xi->m[2] = iTu * r->nZ + iZl;
  xi->m[3] = iTu * r->nZ + iZu;
}

static const double *Crow(const orc_rom *r, int m, int row) { return r->C + ((size_t)m * r->nz + row) * (r->n + 1); }
static double Dval(const orc_rom *r, int m, int row) { return r->D[(size_t)m * r->nz + row]; }

/* OB_step simStep; returns Vcell */
double orc_plant_step(const orc_ctx *X, orc_cell *s, double Iapp) {
  const orc_rom *r = X->r;
  const orc_ind *ix = &X->ix;
  const orc_electrode *en = &r->neg, *ep = &r->pos;
  double T = s->Tc + 273.15;
  double F = r->F, R = r->R, Q = r->Q, Rc = r->Rc;
  double Cdleffn = fCdl(r, en, s->SOC0n, T), Cdleffp = fCdl(r, ep, s->SOC0p, T); /* OB_step.m:212-219 */
  double SOCnAvg = s->SOCnAvg, SOCpAvg = s->SOCpAvg;
  double negSOC = SOCnAvg, posSOC = SOCpAvg;
  double cellSOC = (SOCnAvg - en->theta0) / (en->theta100 - en->theta0);
  double dUn = fdUocp(r, en, SOCnAvg, T), dUp = fdUocp(r, ep, SOCpAvg, T);
  double dQn = fabs(en->theta100 - en->theta0), dQp = fabs(ep->theta100 - ep->theta0);
  double res0n = -dQn / (3600 * Q - Cdleffn * dQn * dUn);
  double res0p = dQp / (3600 * Q - Cdleffp * dQp * dUp);
  SOCnAvg = SOCnAvg + res0n * Iapp * r->Ts;
  SOCpAvg = SOCpAvg + res0p * Iapp * r->Ts;
  if (SOCnAvg < 0) SOCnAvg = 0;
  if (SOCnAvg > 1) SOCnAvg = 1;
  if (SOCpAvg < 0) SOCpAvg = 0;
  if (SOCpAvg > 1) SOCpAvg = 1;
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (r->nZ > 1) {
    int a, b;
    two_nearest(X->Zpts, r->nZ, cellSOC, &a, &b);
    iZu = a > b ? a : b; iZl = a < b ? a : b;
  }
  if (r->nT > 1) {
    int a, b;
    two_nearest(X->Tpts, r->nT, T, &a, &b);
    iTu = a > b ? a : b; iTl = a < b ? a : b;
  }
  double Zu = X->Zpts[iZu], Zl = X->Zpts[iZl], Tu = X->Tpts[iTu], Tl = X->Tpts[iTl];
  int mm[4] = {iTl * r->nZ + iZl, iTl * r->nZ + iZu, iTu * r->nZ + iZl, iTu * r->nZ + iZu};
  enum { R_IFDL0, R_IFDL3, R_IF0, R_IF3, R_TH0, R_TH3, R_TE1, R_TEE, R_PHIE, NR };
  int rows[NR] = {ix->Ifdl0, ix->Ifdl3, ix->If0, ix->If3, ix->Thetass0, ix->Thetass3, ix->Thetae1, ix->ThetaeE, ix->PhieE};
  double y[4][NR];
  for (int j = 0; j < 4; ++j)
    for (int q = 0; q < NR; ++q) {
      const double *c = Crow(r, mm[j], rows[q]);
      const double *x = s->bigX + (size_t)mm[j] * (NX + 1);
      double acc = 0.0;
      for (int k = 0; k <= NX; ++k) acc = acc + c[k] * x[k]; /* res0 column kept: rows are not Phise */
      y[j][q] = acc + Dval(r, mm[j], rows[q]) * Iapp;
    }
  for (int m = 0; m < X->NM; ++m)
    for (int k = 0; k <= NX; ++k) {
      double *x = s->bigX + (size_t)m * (NX + 1) + k;
      *x = fma(r->A[(size_t)m * (NX + 1) + k], *x, Iapp);  /* OB_step.m:278, explicit fma */
    }
  double aZ = 0.0, aT = 0.0;
  if (Zu != Zl) aZ = (cellSOC - Zl) / (Zu - Zl);
  if (Tu != Tl) aT = (T - Tl) / (Tu - Tl);
  double yk[NR];
  for (int q = 0; q < NR; ++q)
    yk[q] = (1 - aT) * ((1 - aZ) * y[0][q] + aZ * y[1][q]) + aT * ((1 - aZ) * y[2][q] + aZ * y[3][q]);
  double th0 = fmin(fmax(yk[R_TH0] + s->SOC0n, 1e-6), 1 - 1e-6);
  double th3 = fmin(fmax(yk[R_TH3] + s->SOC0p, 1e-6), 1 - 1e-6);
  double te1 = fmax(yk[R_TE1] + 1, 1e-6);
  double teE = fmax(yk[R_TEE] + 1, 1e-6);
  double k0n = fk0(r, en, negSOC, T), k0p = fk0(r, ep, posSOC, T); /* OB_step.m:329-330 */
  double i0n = k0n * msqrt(te1 * (1 - th0) * th0);
  double i0p = k0p * msqrt(teE * (1 - th3) * th3);
  double negEta0 = 2 * R * T / F * dasinh(yk[R_IF0] / (2 * i0n));
  double posEta3 = 2 * R * T / F * dasinh(yk[R_IF3] / (2 * i0p));
  double Uocpn0 = fUocp(r, en, th0, T), Uocpp3 = fUocp(r, ep, th3, T);
  double Rfn = fRf(r, en, negSOC, T), Rfp = fRf(r, ep, posSOC, T); /* OB_step.m:339-340 */
  double V = posEta3 - negEta0 + yk[R_PHIE] + Uocpp3 - Uocpn0 + (Rfp * yk[R_IFDL3] - Rfn * yk[R_IFDL0]);
  V = V - Rc * Iapp;
  s->SOCnAvg = SOCnAvg;
  s->SOCpAvg = SOCpAvg;
  return V;
}

/* getVariables (iterEKF.m:259-417); Z has nz entries. Returns Vcell. */
static double get_variables(const orc_ctx *X, orc_cell *s, double ik, const orc_xind *xi, double T, double *Z,
                            double *Zsoc) {
  const orc_rom *r = X->r;
  const orc_ind *ix = &X->ix;
  const orc_electrode *en = &r->neg, *ep = &r->pos;
  int nz = r->nz;
  double xSOC = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q));
  double SOCnAvg = fsoc(r, en, xSOC, T), SOCpAvg = fsoc(r, ep, xSOC, T);
  if (SOCnAvg < 0) { s->warn++; SOCnAvg = 1e-6; }
  if (SOCnAvg > 1) { s->warn++; SOCnAvg = 1 - 1e-6; }
  if (SOCpAvg < 0) { s->warn++; SOCpAvg = 1e-6; }
  if (SOCpAvg > 0.998) { s->warn++; SOCpAvg = 0.998; }
  for (int q = 0; q < nz; ++q) Z[q] = 0.0;
  for (int j = 0; j < 4; ++j) {
    const double *x = X->c->method ? s->xmb : s->xhat + (size_t)xi->m[j] * NX; /* MB: iterEKF.m:314-315 */
    for (int q = 0; q < nz; ++q) {
      const double *c = Crow(r, xi->m[j], q);
      double acc = 0.0;
      for (int k = 0; k < NX; ++k) acc = fma(c[k], x[k], acc);
      double zj = fma(Dval(r, xi->m[j], q), ik, acc);
      Z[q] = fma(zj, xi->g[j], Z[q]);
    }
  }
  double If0 = Z[ix->If0], If3 = Z[ix->If3];
  int any = 0;
  for (int k = 0; k < ix->nNegTh; ++k) { Z[ix->negTh[k]] = Z[ix->negTh[k]] + SOCnAvg; any |= Z[ix->negTh[k]] < 0; }
  if (any) { s->warn++; for (int k = 0; k < ix->nNegTh; ++k) if (Z[ix->negTh[k]] < 0) Z[ix->negTh[k]] = 1e-6; }
  any = 0;
  for (int k = 0; k < ix->nNegTh; ++k) any |= Z[ix->negTh[k]] > 1;
  if (any) { s->warn++; for (int k = 0; k < ix->nNegTh; ++k) if (Z[ix->negTh[k]] > 1) Z[ix->negTh[k]] = 1 - 1e-6; }
  any = 0;
  for (int k = 0; k < ix->nPosTh; ++k) { Z[ix->posTh[k]] = Z[ix->posTh[k]] + SOCpAvg; any |= Z[ix->posTh[k]] < 0; }
  if (any) { s->warn++; for (int k = 0; k < ix->nPosTh; ++k) if (Z[ix->posTh[k]] < 0) Z[ix->posTh[k]] = 1e-6; }
  any = 0;
  for (int k = 0; k < ix->nPosTh; ++k) any |= Z[ix->posTh[k]] > 0.998;
  if (any) { s->warn++; for (int k = 0; k < ix->nPosTh; ++k) if (Z[ix->posTh[k]] > 0.998) Z[ix->posTh[k]] = 0.998; }
  double Un = fUocp(r, en, SOCnAvg, T), Up = fUocp(r, ep, SOCpAvg, T);
  for (int k = 0; k < ix->nNegPhise; ++k) Z[ix->negPhise[k]] = Z[ix->negPhise[k]] + Un;
  for (int k = 0; k < ix->nPosPhise; ++k) Z[ix->posPhise[k]] = Z[ix->posPhise[k]] + Up;
  double PhieTilde3 = Z[ix->PhieE];
  double Phise0 = Z[ix->Phise0];
  for (int k = 0; k < ix->nPhie; ++k) {
    int q = ix->Phie[k];
    if (ix->PhieLoc0[k]) Z[q] = 0 - Phise0;
    else Z[q] = Z[q] - Phise0;
  }
  any = 0;
  for (int k = 0; k < ix->nThetae; ++k) { Z[ix->Thetae[k]] = Z[ix->Thetae[k]] + 1; any |= Z[ix->Thetae[k]] < 0; }
  if (any) { s->warn++; s->status |= ST_ERROR | ST_THETAE_NEG; return NAN; }
  double k0n = fk0(r, en, SOCnAvg, T), k0p = fk0(r, ep, SOCpAvg, T); /* iterEKF.m:392-393 */
  double i0n = k0n * msqrt(Z[ix->Thetae1] * (1 - Z[ix->Thetass0]) * Z[ix->Thetass0]);
  double i0p = k0p * msqrt(Z[ix->ThetaeE] * (1 - Z[ix->Thetass3]) * Z[ix->Thetass3]);
  double negEta0 = 2 * r->R * T / r->F * dasinh(If0 / (2 * i0n));
  double posEta3 = 2 * r->R * T / r->F * dasinh(If3 / (2 * i0p));
  double Uocpn0 = fUocp(r, en, Z[ix->Thetass0], T), Uocpp3 = fUocp(r, ep, Z[ix->Thetass3], T);
  double Rfn = fRf(r, en, SOCnAvg, T), Rfp = fRf(r, ep, SOCpAvg, T); /* iterEKF.m:406-407 */
  double V = posEta3 - negEta0 + PhieTilde3 + Uocpp3 - Uocpn0 + (Rfp * Z[ix->Ifdl3] - Rfn * Z[ix->Ifdl0]);
  for (int k = 0; k < ix->nPosPhis; ++k) Z[ix->posPhis[k]] = Z[ix->posPhis[k]] + V;
  *Zsoc = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q));
  return V;
}

/* getChatV (iterEKF.m:421-519) */
static void get_chat_v(const orc_ctx *X, const orc_cell *s, const orc_xind *xi, const double *Z, double T,
                       double Chat[4][NX], double *Chat0) {
  const orc_rom *r = X->r;
  const orc_ind *ix = &X->ix;
  const orc_electrode *en = &r->neg, *ep = &r->pos;
  double xSOC = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q));
  double SOCnAvg = fsoc(r, en, xSOC, T), SOCpAvg = fsoc(r, ep, xSOC, T); /* iterEKF.m:439-442: unclamped */
  double Rfn = fRf(r, en, SOCnAvg, T), Rfp = fRf(r, ep, SOCpAvg, T);
  double k0n = fk0(r, en, SOCnAvg, T), k0p = fk0(r, ep, SOCpAvg, T);
  double i0n = k0n * msqrt(Z[ix->Thetae1] * (1 - Z[ix->Thetass0]) * Z[ix->Thetass0]);
  double i0p = k0p * msqrt(Z[ix->ThetaeE] * (1 - Z[ix->Thetass3]) * Z[ix->Thetass3]);
  double Rctn = r->R * T / (r->F * i0n), Rctp = r->R * T / (r->F * i0p);
  double dUn0 = fdUocp(r, en, Z[ix->Thetass0], T), dUp3 = fdUocp(r, ep, Z[ix->Thetass3], T);
  for (int j = 0; j < 4; ++j) {
    double g = xi->g[j];
    int m = xi->m[j];
    const double *cIfdl3 = Crow(r, m, ix->Ifdl3), *cIfdl0 = Crow(r, m, ix->Ifdl0), *cIf3 = Crow(r, m, ix->If3),
                 *cIf0 = Crow(r, m, ix->If0), *cPh = Crow(r, m, ix->PhieE), *cT3 = Crow(r, m, ix->Thetass3),
                 *cT0 = Crow(r, m, ix->Thetass0);
    for (int k = 0; k < NX; ++k) {
      double v = Rfp * (g * cIfdl3[k]) - Rfn * (g * cIfdl0[k]);
      v = v + Rctp * (g * cIf3[k]) - Rctn * (g * cIf0[k]);
      v = v + g * cPh[k];
      v = v + (dUp3 * (g * cT3[k]) - dUn0 * (g * cT0[k]));
      Chat[j][k] = v;
    }
  }
  double dn = fsoc(r, en, 1, T) - fsoc(r, en, 0, T), dp = fsoc(r, ep, 1, T) - fsoc(r, ep, 0, T);
  double res0n = -dUn0 * r->Ts * dn / (3600 * r->Q);
  double res0p = -dUp3 * r->Ts * dp / (3600 * r->Q);
  *Chat0 = res0p - res0n;
}

/* ---- 'MB' model blend (iterEKF.m:90-102, 125-128, 160-176, 199-203 and the MB branches of
 * getVariables / getChatV / getChatZ).  State: s->xmb (NX) + s->x0 (integrator), s->Smb. ---- */
#define NA (NX + 1)

/* getChatV 'MB' (iterEKF.m:448-459, 475-479, 489-491, 512-517): sums over the four
 * gamma-weighted corner rows, then the terms, integrator entry last. */
static void get_chat_v_mb(const orc_ctx *X, const orc_cell *s, const orc_xind *xi, const double *Z, double T,
                          double ChV[NA]) {
  const orc_rom *r = X->r;
  const orc_ind *ix = &X->ix;
  const orc_electrode *en = &r->neg, *ep = &r->pos;
  double xSOC = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q)); /* x0 = xhat(end) (iterEKF.m:449-452) */
  double SOCnAvg = fsoc(r, en, xSOC, T), SOCpAvg = fsoc(r, ep, xSOC, T);
  double Rfn = fRf(r, en, SOCnAvg, T), Rfp = fRf(r, ep, SOCpAvg, T);
  double k0n = fk0(r, en, SOCnAvg, T), k0p = fk0(r, ep, SOCpAvg, T);
  double i0n = k0n * msqrt(Z[ix->Thetae1] * (1 - Z[ix->Thetass0]) * Z[ix->Thetass0]);
  double i0p = k0p * msqrt(Z[ix->ThetaeE] * (1 - Z[ix->Thetass3]) * Z[ix->Thetass3]);
  double Rctn = r->R * T / (r->F * i0n), Rctp = r->R * T / (r->F * i0p);
  double dUn0 = fdUocp(r, en, Z[ix->Thetass0], T), dUp3 = fdUocp(r, ep, Z[ix->Thetass3], T);
  const int rows[7] = {ix->Ifdl3, ix->Ifdl0, ix->If3, ix->If0, ix->PhieE, ix->Thetass3, ix->Thetass0};
  for (int k = 0; k < NX; ++k) {
    double sum[7];
    for (int t = 0; t < 7; ++t) {
      double a = 0.0;
      for (int j = 0; j < 4; ++j) a = a + xi->g[j] * Crow(r, xi->m[j], rows[t])[k];
      sum[t] = a;
    }
    double v = Rfp * sum[0] - Rfn * sum[1];
    v = v + Rctp * sum[2] - Rctn * sum[3];
    v = v + sum[4];
    v = v + dUp3 * sum[5] - dUn0 * sum[6];
    ChV[k] = v;
  }
  double dn = fsoc(r, en, 1, T) - fsoc(r, en, 0, T), dp = fsoc(r, ep, 1, T) - fsoc(r, ep, 0, T);
  double res0n = -dUn0 * r->Ts * dn / (3600 * r->Q);
  double res0p = -dUp3 * r->Ts * dp / (3600 * r->Q);
  ChV[NX] = res0p - res0n;
}

static int is_pd_n(int n, const double *a) {
  double l[NA][NA], d[NA];
  for (int j = 0; j < n; ++j) {
    double s = a[j * n + j];
    for (int k = 0; k < j; ++k) s = fma(-(l[j][k] * l[j][k]), d[k], s);
    if (!(s > 0)) return 0;
    d[j] = s;
    double inv = 1.0 / s;
    for (int i = j + 1; i < n; ++i) {
      double t = a[i * n + j];
      for (int k = 0; k < j; ++k) t = fma(-(l[i][k] * l[j][k]), d[k], t);
      l[i][j] = t * inv;
    }
  }
  return 1;
}

/* iterEKF.m:164-173 on the full MB covariance (same polar-factor spelling as orc_meas_cov) */
static void meas_cov_mb(double *S, const double *L, double St, int bump) {
  double P[NA * NA], a[NA * NA], V[NA * NA], w[NA], HH[NA * NA];
  for (int r = 0; r < NA; ++r)
    for (int c = 0; c < NA; ++c) P[r * NA + c] = fma(-(L[r] * St), L[c], S[r * NA + c]);
  for (int r = 0; r < NA; ++r)
    for (int c = 0; c < NA; ++c) a[r * NA + c] = (P[r * NA + c] + P[c * NA + r]) * 0.5;
  if (is_pd_n(NA, a)) {
    memcpy(HH, a, sizeof(HH));
  } else {
    orc_jacobi(NA, a, V, w);
    for (int r = 0; r < NA; ++r)
      for (int c = 0; c < NA; ++c) {
        double acc = 0.0;
        for (int k = 0; k < NA; ++k) acc = acc + (V[r * NA + k] * fabs(w[k])) * V[c * NA + k];
        HH[r * NA + c] = acc;
      }
  }
  for (int r = 0; r < NA; ++r)
    for (int c = r; c < NA; ++c) {
      double v = (((P[r * NA + c] + P[c * NA + r]) + HH[r * NA + c]) + HH[c * NA + r]) / 4.0;
      if (bump) v = v * 2.0;
      S[r * NA + c] = v;
      S[c * NA + r] = v;
    }
}

static double qform_full(const double *S, const double *row) {
  double acc = 0.0;
  for (int c = 0; c < NA; ++c) {
    double t = 0.0;
    for (int k = 0; k < NA; ++k) t = fma(S[k * NA + c], row[k], t);
    acc = fma(t, row[c], acc);
  }
  return acc;
}

static int ekf_step_mb(const orc_ctx *X, orc_cell *s, double vk, double ik, double Tk, double *zk, double *zbk,
                       orc_xind *xo) {
  const orc_rom *r = X->r;
  const orc_cfg *cf = X->c;
  const orc_ind *ix = &X->ix;
  int nz = r->nz;
  double rs = r->Ts / (3600 * r->Q);
  double W = cf->SigmaW;
  orc_xind xi;
  get_xind(X, Tk, s->SOC0 - s->x0 * rs, &xi); /* iterEKF.m:92-93 */
  double amb[NA];
  for (int k = 0; k < NX; ++k) {
    double a = 0.0;
    for (int j = 0; j < 4; ++j) a = a + r->A[(size_t)xi.m[j] * (NX + 1) + k] * xi.g[j];
    amb[k] = a;
  }
  amb[NX] = 1.0;
  for (int k = 0; k < NX; ++k) s->xmb[k] = amb[k] * s->xmb[k] + s->priorI;
  s->x0 = s->x0 + s->priorI;
  for (int p = 0; p < NA; ++p)
    for (int q = 0; q < NA; ++q) s->Smb[p * NA + q] = (amb[p] * s->Smb[p * NA + q]) * amb[q] + W;
  get_xind(X, Tk, s->SOC0 - s->x0 * rs, &xi);
  double Z[256], Zsoc;
  double vhat = get_variables(X, s, ik, &xi, Tk, Z, &Zsoc);
  if (s->status & ST_ERROR) return -1;
  double ChV[NA], L[NA];
  get_chat_v_mb(X, s, &xi, Z, Tk, ChV); /* iterEKF.m:125-128 */
  double St = qform_full(s->Smb, ChV) + cf->SigmaV;
  for (int p = 0; p < NA; ++p) {
    double acc = 0.0;
    for (int k = 0; k < NA; ++k) acc = fma(s->Smb[p * NA + k], ChV[k], acc);
    L[p] = acc / St;
  }
  double res = vk - vhat;
  for (int k = 0; k < NX; ++k) s->xmb[k] = fma(L[k], res, s->xmb[k]);
  s->x0 = fma(L[NX], res, s->x0);
  meas_cov_mb(s->Smb, L, St, res * res > 9 * St);
  get_xind(X, Tk, s->SOC0 - s->x0 * rs, &xi);
  vhat = get_variables(X, s, ik, &xi, Tk, Z, &Zsoc);
  if (s->status & ST_ERROR) return -1;
  for (int q = 0; q < nz; ++q) zk[q] = Z[q];
  zk[nz] = vhat;
  zk[nz + 1] = Zsoc;
  if (zbk) { /* getChatZ 'MB' (iterEKF.m:537-538, 554-558, 575-576, 596-600) + iterEKF.m:199-203 */
    const orc_electrode *en = &r->neg, *ep = &r->pos;
    double ChVz[NA];
    get_chat_v_mb(X, s, &xi, zk, Tk, ChVz);
    double res0n = -r->Ts * (fsoc(r, en, 1, Tk) - fsoc(r, en, 0, Tk)) / (3600 * r->Q);
    double res0p = -r->Ts * (fsoc(r, ep, 1, Tk) - fsoc(r, ep, 0, Tk)) / (3600 * r->Q);
    double xSOC = s->SOC0 - s->x0 * rs;
    double dUn = fdUocp(r, en, fsoc(r, en, xSOC, Tk), Tk), dUp = fdUocp(r, ep, fsoc(r, ep, xSOC, Tk), Tk);
    double Ch[256][NA];
    double c0[256];
    for (int q = 0; q < nz; ++q) {
      for (int k = 0; k < NX; ++k) {
        double a = 0.0;
        for (int j = 0; j < 4; ++j) a = a + xi.g[j] * Crow(r, xi.m[j], q)[k];
        Ch[q][k] = a;
      }
      c0[q] = 0.0;
    }
    for (int t = 0; t < ix->nPosPhis; ++t) {
      int q = ix->posPhis[t];
      for (int k = 0; k < NX; ++k) Ch[q][k] = Ch[q][k] + ChVz[k];
      c0[q] = ChVz[NX];
    }
    for (int k = 0; k < ix->nNegTh; ++k) c0[ix->negTh[k]] = res0n;
    for (int k = 0; k < ix->nPosTh; ++k) c0[ix->posTh[k]] = res0p;
    for (int k = 0; k < ix->nNegPhise; ++k) c0[ix->negPhise[k]] = dUn * res0n;
    for (int k = 0; k < ix->nPosPhise; ++k) c0[ix->posPhise[k]] = dUp * res0p;
    for (int k = 0; k < ix->nPhie; ++k) c0[ix->Phie[k]] = -dUn * res0n;
    for (int t = 0; t < ix->nPhie; ++t) {
      int q = ix->Phie[t];
      for (int k = 0; k < NX; ++k) Ch[q][k] = Ch[q][k] - Ch[ix->Phise0][k];
    }
    for (int q = 0; q < nz; ++q) {
      Ch[q][NX] = c0[q];
      zbk[q] = 3 * msqrt(qform_full(s->Smb, Ch[q]));
    }
    zbk[nz] = 3 * msqrt(qform_full(s->Smb, ChVz));
    zbk[nz + 1] = 3 * msqrt(rs * s->Smb[NA * NA - 1] * rs);
  }
  s->priorI = ik;
  if (xo) *xo = xi;
  return 0;
}

/* iterEKF 'OB' one step.  zk: nz+2, zbk: nz+2 (may be NULL). Returns 0 ok. */
int orc_ekf_step(const orc_ctx *X, orc_cell *s, double vk, double ik, double Tc, double *zk, double *zbk,
                 orc_xind *xo) {
  const orc_rom *r = X->r;
  const orc_cfg *cf = X->c;
  const orc_ind *ix = &X->ix;
  int nz = r->nz;
  if (s->status & ST_ERROR) return -1;
  if (s->warn > cf->max_warn) { s->status |= ST_LOCKOUT | ST_ERROR; return -1; }
  double Tk = Tc > 100 ? Tc : Tc + 273.15;
  if (cf->method) return ekf_step_mb(X, s, vk, ik, Tk, zk, zbk, xo);
  double W = cf->SigmaW;
  for (int m = 0; m < X->NM; ++m) {
    const double *a = r->A + (size_t)m * (NX + 1);
    double *x = s->xhat + (size_t)m * NX;
    double *S = s->S + (size_t)m * NPK;
    /* xhat = A xhat + B i, Sigma = A Sigma A' + SigmaW with A diagonal, as explicit fma:
     * x_e = fma(a_e, x_e, i), S_pq = fma(a_p a_q, S_pq, W) (the kernels' spelling) */
    for (int e = 0; e < NX; ++e) x[e] = fma(a[e], x[e], s->priorI);
    for (int p = 0; p < NX; ++p)
      for (int q = p; q < NX; ++q) S[PK[p][q]] = fma(a[p] * a[q], S[PK[p][q]], W);
  }
  s->x0 = s->x0 + s->priorI;
  s->S0 = s->S0 + W;
  double SOC = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q));
  orc_xind xi;
  get_xind(X, Tk, SOC, &xi);
  double Z[256], Zsoc;
  double vhat = get_variables(X, s, ik, &xi, Tk, Z, &Zsoc);
  if (s->status & ST_ERROR) return -1;
  double ChatV[4][NX], C0;
  get_chat_v(X, s, &xi, Z, Tk, ChatV, &C0);
  const double *S1 = s->S + (size_t)xi.m[0] * NPK;
  double St[4], L[4][NX];
  for (int j = 0; j < 4; ++j) {
    double row[NX];
    for (int c = 0; c < NX; ++c) {
      double acc = 0.0;
      for (int k = 0; k < NX; ++k) acc = fma(S1[PK[k][c]], ChatV[j][k], acc);
      row[c] = acc;
    }
    double acc = 0.0;
    for (int c = 0; c < NX; ++c) acc = fma(row[c], ChatV[j][c], acc);
    St[j] = acc + cf->SigmaV;
    for (int k = 0; k < NX; ++k) L[j][k] = row[k] / St[j]; /* Sigma symmetric: Sigma*c == (c'*Sigma)' */
  }
  double St0 = C0 * s->S0 * C0 + cf->SigmaV;
  double L0 = s->S0 * C0 / St0;
  double res = vk - vhat;
  for (int j = 0; j < 4; ++j) {
    double *x = s->xhat + (size_t)xi.m[j] * NX;
    double *S = s->S + (size_t)xi.m[j] * NPK;
    for (int k = 0; k < NX; ++k) x[k] = fma(L[j][k], res, x[k]);
    orc_meas_cov(S, L[j], St[j], res * res > 9 * St[j]);
  }
  s->x0 = fma(L0, res, s->x0);
  s->S0 = s->S0 - L0 * St0 * L0;
  SOC = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q));
  get_xind(X, Tk, SOC, &xi);
  vhat = get_variables(X, s, ik, &xi, Tk, Z, &Zsoc);
  if (s->status & ST_ERROR) return -1;
  for (int q = 0; q < nz; ++q) zk[q] = Z[q];
  zk[nz] = vhat;
  zk[nz + 1] = Zsoc;
  if (zbk) {
    /* getChatZ (iterEKF.m:523-602) + bounds (iterEKF.m:186-205), diagonal only */
    double ChV[4][NX], ChV0;
    get_chat_v(X, s, &xi, zk, Tk, ChV, &ChV0);
    const orc_electrode *en = &r->neg, *ep = &r->pos;
    double res0n = -r->Ts * (fsoc(r, en, 1, Tk) - fsoc(r, en, 0, Tk)) / (3600 * r->Q);
    double res0p = -r->Ts * (fsoc(r, ep, 1, Tk) - fsoc(r, ep, 0, Tk)) / (3600 * r->Q);
    double xSOC = s->SOC0 - s->x0 * (r->Ts / (3600 * r->Q));
    double dUn = fdUocp(r, en, fsoc(r, en, xSOC, Tk), Tk), dUp = fdUocp(r, ep, fsoc(r, ep, xSOC, Tk), Tk);
    double c0[256];
    for (int q = 0; q < nz; ++q) c0[q] = 0.0;
    for (int k = 0; k < ix->nPosPhis; ++k) c0[ix->posPhis[k]] = ChV0;
    for (int k = 0; k < ix->nNegTh; ++k) c0[ix->negTh[k]] = res0n;
    for (int k = 0; k < ix->nPosTh; ++k) c0[ix->posTh[k]] = res0p;
    for (int k = 0; k < ix->nNegPhise; ++k) c0[ix->negPhise[k]] = dUn * res0n;
    for (int k = 0; k < ix->nPosPhise; ++k) c0[ix->posPhise[k]] = dUp * res0p;
    for (int k = 0; k < ix->nPhie; ++k) c0[ix->Phie[k]] = -dUn * res0n;
    unsigned char isPosPhis[256] = {0}, isPhie[256] = {0};
    for (int k = 0; k < ix->nPosPhis; ++k) isPosPhis[ix->posPhis[k]] = 1;
    for (int k = 0; k < ix->nPhie; ++k) isPhie[ix->Phie[k]] = 1;
    double T1[NPK];
    qform_prep(s->S + (size_t)xi.m[0] * NPK, T1);  /* SigmaX of the first corner (iterEKF.m:191) */
    double SigZ[256], SigV = 0.0;
    for (int q = 0; q < nz; ++q) SigZ[q] = 0.0;
    for (int j = 0; j < 4; ++j) {
      double g = xi.g[j];
      int m = xi.m[j];
      /* Phise0 row of Chat{j} after the posPhis additions */
      double cph0[NX];
      for (int k = 0; k < NX; ++k) {
        double v = g * Crow(r, m, ix->Phise0)[k];
        if (isPosPhis[ix->Phise0]) v = v + ChV[j][k];
        cph0[k] = v;
      }
      for (int q = 0; q < nz; ++q) {
        double row[NX];
        for (int k = 0; k < NX; ++k) {
          double v = isPosPhis[q] ? fma(g, Crow(r, m, q)[k], ChV[j][k]) : g * Crow(r, m, q)[k];
          if (isPhie[q]) v = v - cph0[k];
          row[k] = v;
        }
        SigZ[q] = SigZ[q] + qform(T1, row);
      }
      SigV = SigV + qform(T1, ChV[j]);
    }
    for (int q = 0; q < nz; ++q) SigZ[q] = SigZ[q] + (c0[q] * s->S0) * c0[q];
    SigV = SigV + ChV0 * s->S0 * ChV0;
    double rr = -r->Ts / (3600 * r->Q);
    double SigSOC = rr * s->S0 * rr;
    for (int q = 0; q < nz; ++q) zbk[q] = 3 * msqrt(SigZ[q]);
    zbk[nz] = 3 * msqrt(SigV);
    zbk[nz + 1] = 3 * msqrt(SigSOC);
  }
  s->priorI = ik;
  if (xo) *xo = xi;
  return 0;
}

typedef struct {
  double a[NX + 1], Csoc[NX + 1], Dsoc, Cv[NX + 1], Dv, Cphi[NX + 1], Dphi, bv, bphi, xhat[NX + 1];
} orc_lin;
_Static_assert(sizeof(orc_lin) == 35 * sizeof(double), "orc_lin is the 35-double record");

/* EKFmatsHandler.m:26-114 */
void orc_mats_handler(const orc_ctx *X, const orc_cell *s, const orc_xind *xi, const double *zk, double Tc,
                      orc_lin *L) {
  const orc_rom *r = X->r;
  const orc_ind *ix = &X->ix;
  const orc_electrode *en = &r->neg, *ep = &r->pos;
  int imax = 0;
  for (int j = 1; j < 4; ++j)
    if (xi->g[j] > xi->g[imax] || (xi->g[imax] != xi->g[imax] && xi->g[j] == xi->g[j])) imax = j;
  int m = xi->m[imax];
  for (int k = 0; k < NX; ++k) { L->xhat[k] = s->xhat[(size_t)m * NX + k]; L->a[k] = r->A[(size_t)m * (NX + 1) + k]; }
  L->xhat[NX] = X->c->method ? s->x0 : 0.0; /* ekfData.xhat(end): never updated in 'OB' */
  L->a[NX] = 1.0;
  double rr = -r->Ts / (3600 * r->Q);
  for (int k = 0; k <= NX; ++k) L->Csoc[k] = 0.0;
  L->Csoc[NX] = rr;
  L->Dsoc = 0.0;
  double TK = Tc + 273.15;
  double SOCavg = zk[r->nz + 1];
  double SOCnAvg = fsoc(r, en, SOCavg, TK), SOCpAvg = fsoc(r, ep, SOCavg, TK); /* EKFmatsHandler.m:57-58 */
  double k0n = fk0(r, en, SOCnAvg, TK), k0p = fk0(r, ep, SOCpAvg, TK);
  double i0n = k0n * msqrt(zk[ix->Thetae1] * (1 - zk[ix->Thetass0]) * zk[ix->Thetass0]);
  double i0p = k0p * msqrt(zk[ix->ThetaeE] * (1 - zk[ix->Thetass3]) * zk[ix->Thetass3]);
  double Rfn = fRf(r, en, SOCnAvg, TK), Rfp = fRf(r, ep, SOCpAvg, TK); /* EKFmatsHandler.m:68-69 */
  for (int k = 0; k < NX; ++k)
    L->Cv[k] = Rfp * Crow(r, m, ix->Ifdl3)[k] - Rfn * Crow(r, m, ix->Ifdl0)[k] + Crow(r, m, ix->PhieE)[k];
  L->Cv[NX] = 0.0;
  L->Dv = Rfp * Dval(r, m, ix->Ifdl3) - Rfn * Dval(r, m, ix->Ifdl0) + Dval(r, m, ix->PhieE);
  double Upos = fUocp(r, ep, zk[ix->Thetass3], TK), Uneg = fUocp(r, en, zk[ix->Thetass0], TK);
  double negEta0 = 2 * r->R * TK / r->F * dasinh(zk[ix->If0] / (2 * i0n));
  double posEta3 = 2 * r->R * TK / r->F * dasinh(zk[ix->If3] / (2 * i0p));
  double b_phi = 0.01 * 0;
  L->bv = (Upos - Uneg) + (posEta3 - negEta0) + b_phi;
  L->bphi = fUocp1(r, en, SOCnAvg); /* one-argument call (EKFmatsHandler.m:96) */
  for (int k = 0; k < NX; ++k) L->Cphi[k] = Crow(r, m, ix->negPhise2)[k];
  L->Cphi[NX] = 0.0;
  L->Dphi = Dval(r, m, ix->negPhise2);
}

/* constraintsMPC.m:11-112 -> M (nC x Nc row-major), gam (nC); returns nC.
 * Phis/Gs: mpcData.Phi_soc / G_soc of this step (iterMPC.m:33-34). */
int orc_constraints(const orc_rom *r, const orc_cfg *cf, const orc_lin *L, const double *x /*7*/, double uk_1,
                    double SOCk_1, const double *Phis, const double *Gs, double *M, double *gam) {
  int Np = cf->Np, Nc = cf->Nc, nr = 0;
  const int na = NX + 2;
  if (cf->use_cur) {
    double u_min = -r->Q * cf->Crate; /* initMPC.m:66-67 */
    for (int i = 0; i < Nc; ++i) { /* Cu = tril(ones(Nc)) */
      for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = j <= i ? 1.0 : 0.0;
      gam[nr + i] = (cf->u_max - uk_1) * 1.0;
    }
    nr += Nc;
    for (int i = 0; i < Nc; ++i) {
      for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = -(j <= i ? 1.0 : 0.0);
      gam[nr + i] = -(u_min - uk_1) * 1.0;
    }
    nr += Nc;
    for (int i = 0; i < Nc; ++i) {
      for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = i == j ? 1.0 : 0.0;
      gam[nr + i] = cf->du_max * 1.0;
    }
    nr += Nc;
    for (int i = 0; i < Nc; ++i) {
      for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = -(i == j ? 1.0 : 0.0);
      gam[nr + i] = -cf->du_min * 1.0;
    }
    nr += Nc;
  }
  double Phi[NPMAX * (NX + 2)], G[NPMAX * NCMAX];
  if (cf->use_v) {
    orc_predmat(L->a, L->Cv, L->Dv, Np, Nc, Phi, G);
    for (int i = 0; i < Np; ++i) {
      double acc = 0.0;
      for (int k = 0; k < na; ++k) acc = acc + Phi[i * na + k] * x[k];
      double rhs = acc + L->bv * 1.0;
      for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = G[i * Nc + j];
      gam[nr + i] = cf->v_max - rhs;
    }
    nr += Np;
  }
  if (cf->use_eta) {
    orc_predmat(L->a, L->Cphi, L->Dphi, Np, Nc, Phi, G);
    for (int i = 0; i < Np; ++i) {
      double acc = 0.0;
      for (int k = 0; k < na; ++k) acc = acc + Phi[i * na + k] * x[k];
      double rhs = acc + L->bphi * 1.0;
      for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = -G[i * Nc + j];
      gam[nr + i] = -cf->phise_min + rhs;
    }
    nr += Np;
  }
  double zmax = cf->z_max + cf->z_tol;
  for (int i = 0; i < Np; ++i) {
    double acc = 0.0;
    for (int k = 0; k < na; ++k) acc = acc + Phis[i * na + k] * x[k];
    double rhs = acc + SOCk_1 * 1.0;
    for (int j = 0; j < Nc; ++j) M[(nr + i) * Nc + j] = Gs[i * Nc + j];
    gam[nr + i] = zmax * 1.0 - rhs;
  }
  nr += Np;
  return nr;
}

typedef struct {
  double uk, J_unc, J_fin, norm_du; /* mpcData.cost (iterMPC.m:89-95) */
  int nexec, nviol;
} orc_mpc_out;

/* iterMPC.m:17-95 (diagnostics :54-60 are out of scope) */
void orc_mpc_step(const orc_rom *r, const orc_cfg *cf, orc_cell *s, const orc_lin *L, double SOCk_1,
                  orc_mpc_out *o) {
  int Np = cf->Np, Nc = cf->Nc;
  const int na = NX + 2;
  double dx[NX + 2];
  for (int k = 0; k <= NX; ++k) dx[k] = L->xhat[k];
  dx[NX + 1] = s->uk_1;
  double Phis[NPMAX * (NX + 2)], Gs[NPMAX * NCMAX];
  orc_predmat(L->a, L->Csoc, L->Dsoc, Np, Nc, Phis, Gs);
  double e[NPMAX];
  for (int i = 0; i < Np; ++i) {
    double acc = 0.0;
    for (int k = 0; k < na; ++k) acc = acc + Phis[i * na + k] * dx[k];
    e[i] = cf->ref * 1.0 - acc;
  }
  double F[NCMAX];
  for (int j = 0; j < Nc; ++j) {
    double acc = 0.0;
    for (int i = 0; i < Np; ++i) acc = acc + (-2 * Gs[i * Nc + j]) * e[i];
    F[j] = acc;
  }
  double GtG[NCMAX * NCMAX];
  for (int a = 0; a < Nc; ++a)
    for (int b = 0; b < Nc; ++b) {
      double acc = 0.0;
      for (int i = 0; i < Np; ++i) acc = acc + Gs[i * Nc + a] * Gs[i * Nc + b];
      GtG[a * Nc + b] = acc;
    }
  double smin = orc_sigma_min(Nc, GtG);
  double nF = 0.0;
  for (int j = 0; j < Nc; ++j) nF = nF + F[j] * F[j];
  nF = sqrt(nF);
  double Ru = (nF / (2 * cf->du_max * sqrt((double)Nc))) - smin;
  double E[NCMAX * NCMAX], mE[NCMAX * NCMAX];
  for (int a = 0; a < Nc; ++a)
    for (int b = 0; b < Nc; ++b) {
      E[a * Nc + b] = 2 * (GtG[a * Nc + b] + Ru * (a == b ? 1.0 : 0.0));
      mE[a * Nc + b] = -E[a * Nc + b];
    }
  double DU[NCMAX];
  lu_solve(Nc, mE, F, DU);
  double Jr[NPMAX];
  for (int i = 0; i < Np; ++i) {
    double acc = 0.0;
    for (int j = 0; j < Nc; ++j) acc = acc + Gs[i * Nc + j] * DU[j];
    Jr[i] = e[i] - acc;
  }
  double J = 0.0, Jq = 0.0;
  for (int i = 0; i < Np; ++i) J = J + Jr[i] * Jr[i];
  for (int c = 0; c < Nc; ++c) {
    double acc = 0.0;
    for (int k = 0; k < Nc; ++k) acc = acc + (Ru * (c == k ? 1.0 : 0.0)) * DU[k];
    Jq = Jq + acc * DU[c];
  }
  o->J_unc = J + Jq;
  double M[NCONMAX * NCMAX], gam[NCONMAX];
  int nC = orc_constraints(r, cf, L, dx, s->uk_1, SOCk_1, Phis, Gs, M, gam);
  int nv = 0;
  for (int i = 0; i < nC; ++i) {
    double acc = 0.0;
    for (int j = 0; j < Nc; ++j) acc = acc + M[i * Nc + j] * DU[j];
    if (acc - gam[i] > 0) nv++;
  }
  o->nexec = 0;
  if (nv > 0) o->nexec = orc_hildreth(Nc, nC, E, F, M, gam, s->lam, cf->maxHild, cf->hild_tol, DU);
  double uk = DU[0] + s->uk_1;
  s->uk_1 = uk;
  o->uk = uk;
  int nviol = 0;
  for (int i = 0; i < nC; ++i) {
    double acc = 0.0;
    for (int j = 0; j < Nc; ++j) acc = acc + M[i * Nc + j] * DU[j];
    if (acc - gam[i] > 1e-9) nviol++;
  }
  o->nviol = nviol;
  for (int i = 0; i < Np; ++i) {
    double acc = 0.0;
    for (int j = 0; j < Nc; ++j) acc = acc + Gs[i * Nc + j] * DU[j];
    Jr[i] = e[i] - acc;
  }
  J = 0.0; Jq = 0.0;
  for (int i = 0; i < Np; ++i) J = J + Jr[i] * Jr[i];
  for (int c = 0; c < Nc; ++c) {
    double acc = 0.0;
    for (int k = 0; k < Nc; ++k) acc = acc + (Ru * (c == k ? 1.0 : 0.0)) * DU[k];
    Jq = Jq + acc * DU[c];
  }
  o->J_fin = J + Jq;
  double s2 = 0.0; /* norm(DU,2) (iterMPC.m:92) as the square root of the sequential sum */
  for (int j = 0; j < Nc; ++j) s2 = s2 + DU[j] * DU[j];
  o->norm_du = sqrt(s2);
}

/* iterMPC.m:17-95 on given EKFmatsHandler records (the 35-double layout of orc_lin,
 * include/mpcekf.h MPCEKF_LIN_*): open-loop parity of the MPC stage.  uk_1 and lam
 * ([n][nC]) are the mpcData state in and out. */
int orc_mpc_lin(const orc_rom *r, const orc_cfg *c, int n, const double *lin, const double *soc_k1, double *uk_1,
                double *lam, double *uk, int32_t *nexec) {
  if (c->Np > NPMAX || c->Nc > NCMAX) return -10;
  const int nC = (c->use_cur ? 4 * c->Nc : 0) + (c->use_v ? c->Np : 0) + (c->use_eta ? c->Np : 0) + c->Np;
  for (int i = 0; i < n; ++i) {
    orc_cell s;
    memset(&s, 0, sizeof s);
    s.uk_1 = uk_1[i];
    for (int j = 0; j < nC; ++j) s.lam[j] = lam[(size_t)i * nC + j];
    orc_lin L;
    memcpy(&L, lin + (size_t)i * 35, sizeof L);
    orc_mpc_out o;
    orc_mpc_step(r, c, &s, &L, soc_k1[i], &o);
    uk[i] = o.uk;
    nexec[i] = o.nexec;
    uk_1[i] = s.uk_1;
    for (int j = 0; j < nC; ++j) lam[(size_t)i * nC + j] = s.lam[j];
  }
  return 0;
}

/* ----------------------------------------------------------------------- */
/* driver                                                                   */
/* ----------------------------------------------------------------------- */
static int ctx_init(orc_ctx *X, const orc_rom *r, const orc_cfg *c) {
  X->r = r;
  X->c = c;
  X->NM = r->nT * r->nZ;
  if (r->n != NX || r->nz > 256 || r->nT > 64 || r->nZ > 64 || c->Np > NPMAX || c->Nc > NCMAX) return -10;
  for (int t = 0; t < r->nT; ++t) X->Tpts[t] = r->T_degC[t] + 273.15;
  for (int z = 0; z < r->nZ; ++z) X->Zpts[z] = r->SOC_pct[z] / 100;
  return orc_resolve(r, &X->ix);
}

static void init_cell(const orc_ctx *X, orc_cell *s, double soc0, double tc) {
  const orc_rom *r = X->r;
  const orc_cfg *c = X->c;
  size_t NM = (size_t)X->NM;
  memset(s->bigX, 0, sizeof(double) * NM * (NX + 1));
  memset(s->xhat, 0, sizeof(double) * NM * NX);
  for (size_t m = 0; m < NM; ++m)
    for (int p = 0; p < NX; ++p)
      for (int q = p; q < NX; ++q) s->S[m * NPK + PK[p][q]] = p == q ? c->SigmaX0[p] : 0.0;
  double Tk1 = tc + 273.15; /* OB_step.m:63-65 */
  s->SOC0n = fsoc(r, &r->neg, soc0 / 100, Tk1);
  s->SOC0p = fsoc(r, &r->pos, soc0 / 100, Tk1);
  s->SOCnAvg = s->SOC0n;
  s->SOCpAvg = s->SOC0p;
  s->Tc = tc;
  s->x0 = 0.0;
  s->S0 = c->SigmaX0[NX];
  for (int p = 0; p < NX; ++p) s->xmb[p] = 0.0;
  for (int p = 0; p <= NX; ++p)
    for (int q = 0; q <= NX; ++q) s->Smb[p * (NX + 1) + q] = p == q ? c->SigmaX0[p] : 0.0;
  s->priorI = 0.0;
  s->SOC0 = soc0 / 100;
  s->warn = 0;
  s->status = 0;
  s->uk_1 = 0.0;
  s->uk = 0.0;
  for (int i = 0; i < NCONMAX; ++i) s->lam[i] = 0.0;
}

/* One closed-loop step of runMPC.m:84-111 for one cell. */
/* Per-step diagnostics of runMPC.m:106-111 and mpcData.cost (iterMPC.m:89-95). */
typedef struct {
  double *x;                       /* [nsteps][ncells][6]    x_store (EKFmatsHandler xhat) */
  double *zk, *zbk;                /* [nsteps][ncells][nz+2] zkEst, zkBound                */
  double *J_unc, *J_fin, *norm_du; /* [nsteps][ncells]       J_uncon, J_final, norm_DU     */
  int32_t *nviol;                  /* [nsteps][ncells]       viol                          */
  const double *tc;                /* [nsteps][ncells] INPUT: TC of each step (degC), or NULL */
} orc_traj;

static void cell_step(const orc_ctx *X, orc_cell *s, double *u, double *v, double *soc, double *phise, int *nexec,
                      double *zk_out, double *zbk_out, orc_mpc_out *mo, double *x_out) {
  const orc_rom *r = X->r;
  int nz = r->nz;
  mo->J_unc = mo->J_fin = mo->norm_du = mo->uk = NAN;
  mo->nviol = 0;
  if (x_out) for (int q = 0; q <= NX; ++q) x_out[q] = NAN;
  if (s->status & ST_ERROR) {
    *u = *v = *soc = *phise = NAN;
    *nexec = 0;
    if (zk_out) for (int q = 0; q < nz + 2; ++q) zk_out[q] = NAN;
    if (zbk_out) for (int q = 0; q < nz + 2; ++q) zbk_out[q] = NAN;
    return;
  }
  double ukin = s->uk;
  double V = orc_plant_step(X, s, ukin);
  double zk[258], zbk[258];
  orc_xind xi;
  if (orc_ekf_step(X, s, V, ukin, s->Tc, zk, zbk_out ? zbk : NULL, &xi) != 0) {
    *u = *v = *soc = *phise = NAN;
    *nexec = 0;
    if (zk_out) for (int q = 0; q < nz + 2; ++q) zk_out[q] = NAN;
    if (zbk_out) for (int q = 0; q < nz + 2; ++q) zbk_out[q] = NAN;
    s->uk = NAN;
    return;
  }
  orc_lin L;
  orc_mats_handler(X, s, &xi, zk, s->Tc, &L);
  double acc = 0.0;
  for (int k = 0; k <= NX; ++k) acc = acc + L.Cphi[k] * L.xhat[k];
  double ph = acc + ukin * L.Dphi + L.bphi;
  orc_mpc_out o;
  orc_mpc_step(r, X->c, s, &L, zk[nz + 1], &o);
  *mo = o;
  if (x_out) for (int q = 0; q <= NX; ++q) x_out[q] = L.xhat[q];
  s->uk = o.uk;
  *u = o.uk;
  *v = V;
  *soc = zk[nz + 1];
  *phise = ph;
  *nexec = o.nexec;
  if (zk_out) for (int q = 0; q < nz + 2; ++q) zk_out[q] = zk[q];
  if (zbk_out) for (int q = 0; q < nz + 2; ++q) zbk_out[q] = zbk[q];
}

/* Batched closed loop: outputs are [nsteps][ncells]; zk/zbk (optional) are
 * the LAST step's [ncells][nz+2].  Returns 0 on success. */
int orc_run_traj(const orc_rom *r, const orc_cfg *c, int ncells, const double *soc0, const double *tc, int nsteps,
                 double *u, double *v, double *soc, double *phise, int32_t *nexec, int32_t *status, double *zk,
                 double *zbk, const orc_traj *tr, int nthreads) {
  orc_ctx X;
  int rc = ctx_init(&X, r, c);
  if (rc) return rc;
  size_t NM = (size_t)X.NM;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int i = 0; i < ncells; ++i) {
    orc_cell s;
    s.bigX = (double *)malloc(sizeof(double) * NM * (NX + 1));
    s.xhat = (double *)malloc(sizeof(double) * NM * NX);
    s.S = (double *)malloc(sizeof(double) * NM * NPK);
    init_cell(&X, &s, soc0[i], tc[i]);
    for (int k = 0; k < nsteps; ++k) {
      size_t o = (size_t)k * ncells + i;
      int ne;
      int last = k == nsteps - 1;
      const size_t nzz = (size_t)r->nz + 2;
      double *zko = (tr && tr->zk) ? tr->zk + o * nzz : (zk && last) ? zk + (size_t)i * nzz : NULL;
      double *zbo = (tr && tr->zbk) ? tr->zbk + o * nzz : (zbk && last) ? zbk + (size_t)i * nzz : NULL;
      orc_mpc_out mo;
      if (tr && tr->tc) s.Tc = tr->tc[o]; /* runMPC.m:85-92: the step's TC for all three calls */
      cell_step(&X, &s, &u[o], &v[o], &soc[o], &phise[o], &ne, zko, zbo, &mo,
                (tr && tr->x) ? tr->x + o * (NX + 1) : NULL);
      if (tr && tr->zk && zk && last) memcpy(zk + (size_t)i * nzz, zko, nzz * sizeof(double));
      if (tr && tr->zbk && zbk && last) memcpy(zbk + (size_t)i * nzz, zbo, nzz * sizeof(double));
      if (tr && tr->J_unc) tr->J_unc[o] = mo.J_unc;
      if (tr && tr->J_fin) tr->J_fin[o] = mo.J_fin;
      if (tr && tr->norm_du) tr->norm_du[o] = mo.norm_du;
      if (tr && tr->nviol) tr->nviol[o] = mo.nviol;
      nexec[o] = ne;
    }
    status[i] = s.status;
    free(s.bigX);
    free(s.xhat);
    free(s.S);
  }
  return 0;
}

/* Batched closed loop: outputs are [nsteps][ncells]; zk/zbk (optional) are the LAST
 * step's [ncells][nz+2]. */
int orc_run(const orc_rom *r, const orc_cfg *c, int ncells, const double *soc0, const double *tc, int nsteps,
            double *u, double *v, double *soc, double *phise, int32_t *nexec, int32_t *status, double *zk,
            double *zbk, int nthreads) {
  return orc_run_traj(r, c, ncells, soc0, tc, nsteps, u, v, soc, phise, nexec, status, zk, zbk, NULL, nthreads);
}

int orc_version(void) { return 3; }
