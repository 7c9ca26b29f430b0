// mpcekf_kernels.hip -- gfx950 kernels of the batched MPC+EKF control step.
//
// Work mapping (DESIGN.md "Kernels"):
//   k_plant  lane-per-cell   OB_step.m:188-357 minus the all-model advance
//   k_bulk   block-streaming OB_step.m:278 (bigX = bigA.*bigX + Iapp) and the
//                            all-model EKF time update iterEKF.m:73-84, over the
//                            whole cell batch: the HBM-bound part
//   k_cell   lane-per-cell   iterEKF.m:85-210 (4-corner measurement update),
//                            EKFmatsHandler.m, predMat.m, constraintsMPC.m,
//                            iterMPC.m and hildreth.m for one cell per lane
// The ROM (C/D rows, diag(A), OCP tables) is staged once per workgroup in LDS.
// Arithmetic follows the defined order of oracle/mpcekf_oracle.c (sequential
// sums from +0.0, no contraction, asinh spelled out as dasinh), so results match
// it bit-for-bit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>

#include "mpcekf_kernels.hpp"
#include "mpcekf_mpc.hpp"

#pragma clang fp contract(off)

namespace mk {

constexpr int NP = 5;                  // compiled horizon (runMPC.m:28)
constexpr int NC = 2;                  // compiled control horizon (runMPC.m:29)
constexpr int NCON = 4 * NC + 3 * NP;  // constraint rows (constraintsMPC.m)

// k_cell build options (A/B knobs; the defaults are the measured best):
// MPCEKF_REC_ONCE: corners whose whole record (xhat and Sigma) is read with the first
// read; the others read Sigma at their update.  1: corner 0's Sigma is what the gains
// use first; 2..4 hold more Sigma in registers and spill (measured no faster).
// MPCEKF_CELL_OUTLINE: the Jacobi symmetrisation as a call instead of inline.
#ifndef MPCEKF_S_AHEAD  // k_cell: corner j+1's Sigma loaded before corner j's record store (§4.2)
#define MPCEKF_S_AHEAD 1
#endif
#ifndef MPCEKF_RING_LATE  // k_cell: the plant's ring stores after the cell's last load (§4.2)
#define MPCEKF_RING_LATE 1
#endif
#ifndef MPCEKF_PLANT_STORE_LATE  // k_cell: the plant's state stores after the cell's last load
#define MPCEKF_PLANT_STORE_LATE 0
#endif
#ifndef MPCEKF_REC_ONCE
#define MPCEKF_REC_ONCE 1
#endif
#ifndef MPCEKF_CELL_OUTLINE
#define MPCEKF_CELL_OUTLINE false
#endif
// k_flush: the next cell's loads issued before this cell's replay
#ifndef MPCEKF_FLUSH_PF
#define MPCEKF_FLUSH_PF 1
#endif
// k_hild: rows of LDS operand prefetch in the fast sweep
#ifndef MPCEKF_HILD_PF
#define MPCEKF_HILD_PF 3
#endif
#ifndef MPCEKF_HILD_REGROWS  // k_hild: the constant rows' X / H_ii slots in registers
#define MPCEKF_HILD_REGROWS 1
#endif
#ifndef MPCEKF_FLUSH_COAL  // k_flush_coal (coalesced chunks, NM <= 64): measured slower, off
#define MPCEKF_FLUSH_COAL 0
#endif
// k_hild finishes its slow lanes itself (no k_hild_slow launch).  Off: the exact-rule
// path's registers moved the fast sweep's allocation (AGPRs 34 -> 242) and k_hild took
// 89.5 instead of ~75 us, more than the ~5 us a k_hild_slow launch costs (r04g A/B)
#ifndef MPCEKF_HILD_INLINE_SLOW
#define MPCEKF_HILD_INLINE_SLOW 0
#endif
#ifndef MPCEKF_HILD_NEXTV  // k_hild: the next sweep's v accumulated in the row loop
#define MPCEKF_HILD_NEXTV 1
#endif
// v3 lookups without branches (NaN theta, Ea = 0 and dexp's special cases by selects): one
// basic block per lookup, so neighbouring lookups' L2 loads can overlap; quintic k_cell 45.3k
// -> 43.6k instructions, 1,084 -> 837 branches, same-box 155.3 / 148.0 -> 151.9 / 147.7 us
// (profiles/r05h_ab_branchfree.txt)
#ifndef MPCEKF_PL_BRANCHFREE
#define MPCEKF_PL_BRANCHFREE 1
#endif

// Section timestamps of k_cell for profiling builds (-DMPCEKF_STAMPS); compiled out otherwise.
#ifdef MPCEKF_STAMPS
#define STAMP(i)                                                                          \
  do {                                                                                    \
    if (io.stamps) io.stamps[(size_t)(i) * s.n + c] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#define STAMPP(i)                                                                                  \
  do {                                                                                             \
    if (s.stamps) s.stamps[(size_t)(12 + (i)) * s.n + c] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#define STAMPP(i) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ int pk(int r, int c) {
  // packed upper-triangular index, row-major over r <= c
  return r <= c ? r * NX - (r * (r - 1)) / 2 + (c - r) : c * NX - (c * (c - 1)) / 2 + (r - c);
}

// Defined asinh (the plant/EKF overpotential, OB_step.m:333-334, iterEKF.m:400-401,
// EKFmatsHandler.m:88-89).  Neither ocml's nor glibc's asinh is correctly rounded, so
// the kernels and oracle/mpcekf_oracle.c (orc_asinh) both evaluate this spelling: a
// reduction to log(u) + c with u = 2^k m, m in (sqrt(2)/2, sqrt(2)], and the classic
// minimax series in s = f / (2 + f), f = m - 1 (Lg1..Lg7, fdlibm's public
// coefficients).  Only +, -, *, /, sqrt and fma: correctly rounded on both sides.
namespace dm {
constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
constexpr double LN2 = 6.93147180559945286227e-01;
constexpr double LG1 = 6.666666666666735130e-01, LG2 = 3.999999999940941908e-01, LG3 = 2.857142874366239149e-01,
                 LG4 = 2.222219843214978396e-01, LG5 = 1.818357216161805012e-01, LG6 = 1.531383769920937332e-01,
                 LG7 = 1.479819860511658591e-01;
constexpr double SQRT2 = 1.4142135623730951;
// log(u) + c for a finite u >= 1; c is the relative correction (u_true - u) / u
__device__ __forceinline__ double log_core(double u, double c) {
  unsigned long long b = (unsigned long long)__double_as_longlong(u);
  int k = (int)(b >> 52) - 1023;
  double m = __longlong_as_double((long long)((b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL));
  if (m > SQRT2) { m = 0.5 * m; k = k + 1; }
  double f = m - 1.0;
  double s = f / (2.0 + f);
  double z = s * s;
  double w = z * z;
  double t1 = w * (LG2 + w * (LG4 + w * LG6));
  double t2 = z * (LG1 + w * (LG3 + w * (LG5 + w * LG7)));
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  double dk = (double)k;
  return dk * LN2_HI - ((hfsq - (s * (hfsq + R) + (dk * LN2_LO + c))) - f);
}
}  // namespace dm
__device__ __forceinline__ double dasinh(double x) {
  double a = fabs(x);
  if (!(a < __builtin_inf())) return x + x;  // NaN, +-inf
  if (a < 0x1p-28) return x;
  double t;
  if (a > 0x1p28) {
    t = dm::log_core(a, 0.0) + dm::LN2;
  } else if (a > 2.0) {
    t = dm::log_core(2.0 * a + 1.0 / (sqrt(fma(a, a, 1.0)) + a), 0.0);
  } else {  // log1p(a + a^2 / (1 + sqrt(1 + a^2)))
    double a2 = a * a;
    double xx = a + a2 / (1.0 + sqrt(1.0 + a2));
    double u = 1.0 + xx;
    double c = (xx - (u - 1.0)) / u;
    t = dm::log_core(u, c);
  }
  return x < 0 ? -t : t;
}

// v from the quad lane selected by DPP quad_perm control CTRL.
template <int CTRL>
__device__ __forceinline__ double qperm(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
template <int Q>
__device__ __forceinline__ double qbc(double v) {  // lane Q's v in every lane of the quad
  return qperm<Q | (Q << 2) | (Q << 4) | (Q << 6)>(v);
}
__device__ __forceinline__ double shfl64(double v, int lane) {  // v of lane (runtime), ds_bpermute
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(lane << 2, (int)b);
  const int hi = __builtin_amdgcn_ds_bpermute(lane << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

__device__ __forceinline__ double tabi(const double *t, int n, double x) {
  if (x != x) return __builtin_nan("");
  double xc = fmin(fmax(x, 0.0), 1.0);
  double tt = xc * (double)(n - 1);
  int i = (int)floor(tt);
  if (i > n - 2) i = n - 2;
  double f = tt - (double)i;
  return t[i] + f * (t[i + 1] - t[i]);
}
// ABI v3 polynomial row (include/mpcekf.h tab_npoly): theta's interval i and s = t - i as
// in tabi, then Horner (fma) over the interval's 6 coefficients (a cubic's upper two are 0),
// read from the global table (L2-resident) as three 16-byte loads.  oracle: tab_poly.
// Horner with explicit fma (correctly rounded here and on the host: oracle tab_poly)
__device__ __forceinline__ double horner6(const double2 c01, const double2 c23, const double2 c45, double s) {
  double v = c45.y;
  v = __builtin_fma(s, v, c45.x);
  v = __builtin_fma(s, v, c23.y);
  v = __builtin_fma(s, v, c23.x);
  v = __builtin_fma(s, v, c01.y);
  return __builtin_fma(s, v, c01.x);
}
__device__ __forceinline__ int tab_interval(int n, double x, double &s) {
  double xc = fmin(fmax(x, 0.0), 1.0);
  double tt = xc * (double)(n - 1);
  int i = (int)floor(tt);
  if (i > n - 2) i = n - 2;
  s = tt - (double)i;
  return i;
}
// one row: interval i's coefficients at c + i * istride
__device__ __forceinline__ double tabp(const double *c, int n, double x, int istride) {
#if !MPCEKF_PL_BRANCHFREE
  if (x != x) return __builtin_nan("");
#endif
  double s;
  const int i = tab_interval(n, x, s);  // a NaN x: interval 0 (fmax), the NaN selected below
  const double2 *p = reinterpret_cast<const double2 *>(c + (size_t)i * istride);
  const double v = horner6(p[0], p[1], p[2], s);
  return (MPCEKF_PL_BRANCHFREE && x != x) ? __builtin_nan("") : v;
}
// two adjacent rows of interval i (the T bracket): a from c + i * istride, b KPOLY after
__device__ __forceinline__ void tabp2(const double *c, int n, double x, int istride, double &a, double &b,
                                      int ro = KPOLY) {
#if !MPCEKF_PL_BRANCHFREE
  if (x != x) {
    a = b = __builtin_nan("");
    return;
  }
#endif
  double s;
  const int i = tab_interval(n, x, s);
  const double2 *p = reinterpret_cast<const double2 *>(c + (size_t)i * istride);
  const double2 *q = reinterpret_cast<const double2 *>(c + (size_t)i * istride + ro);
  const double2 a01 = p[0], a23 = p[1], a45 = p[2], b01 = q[0], b23 = q[1], b45 = q[2];
  a = horner6(a01, a23, a45, s);
  b = horner6(b01, b23, b45, s);
  if (MPCEKF_PL_BRANCHFREE && x != x) a = b = __builtin_nan("");
}
// ABI v4 rows on a function's own theta nodes (include/mpcekf.h node / node_p): the segment
// k = #{j in 1..m-2 : x_j <= theta} (oracle node_poly) from the function's uniform bucket map
// (host build_rom: nu buckets over [0, 1], nu a power of two, each bucket holding at most
// one interior node; entry u = (k of u / nu, x_k, x_k+1 or +inf)): floor(theta nu) is exact,
// so the bucket's left edge lies at or below theta and one compare with x_k+1 finishes the
// search.  s = theta - x_k, then Horner over the segment's 6 coefficients as tabp2.
__device__ __forceinline__ void tabn2(const double *c, const double *map, int nu, double x, int istride, double &a,
                                      double &b, int ro) {
  const double xc = fmin(fmax(x, 0.0), 1.0);  // NaN x: 0 (fmax), the NaN selected below
  int u = (int)floor(xc * (double)nu);
  u = u > nu - 1 ? nu - 1 : u;
  const double2 *m = reinterpret_cast<const double2 *>(map + (size_t)u * KMAP);
  const double2 m0 = m[0], m1 = m[1];
  const bool up = xc >= m1.x;
  const int i = (int)m0.x + (up ? 1 : 0);
  const double s = xc - (up ? m1.x : m0.y);
  const double2 *p = reinterpret_cast<const double2 *>(c + (size_t)i * istride);
  const double2 *q = reinterpret_cast<const double2 *>(c + (size_t)i * istride + ro);
  const double2 a01 = p[0], a23 = p[1], a45 = p[2], b01 = q[0], b23 = q[1], b45 = q[2];
  a = horner6(a01, a23, a45, s);
  b = horner6(b01, b23, b45, s);
  if (x != x) a = b = __builtin_nan("");
}
// Defined exp of the v3 Arrhenius factor (oracle/mpcekf_oracle.c orc_exp, rom.py dexp):
// x = k ln2 + r, k = floor(x / ln2 + 1/2), fdlibm's rational form for exp(r); only
// +, -, *, /, floor and ldexp, exact or correctly rounded on both sides.
// MPCEKF_PL_BRANCHFREE: the special cases by selects (the in-range arithmetic unchanged), so
// that a lookup is one basic block
__device__ __forceinline__ double dexp(double x0) {
#if MPCEKF_PL_BRANCHFREE
  const bool nan = x0 != x0, big = x0 > 709.782712893384, small = x0 < -745.1332191019412;
  const double x = (nan || big || small) ? 0.0 : x0;
#else
  const double x = x0;
  if (x != x) return x;
  if (x > 709.782712893384) return __builtin_inf();
  if (x < -745.1332191019412) return 0.0;
#endif
  const double k = floor(x * 1.44269504088896338700e+00 + 0.5);
  const double hi = x - k * dm::LN2_HI;
  const double lo = k * dm::LN2_LO;
  const double r = hi - lo;
  const double t = r * r;
  const double c = r - t * (1.66666666666666019037e-01 +
                            t * (-2.77777777770155933842e-03 +
                                 t * (6.61375632143793436117e-05 +
                                      t * (-1.65339022054652515390e-06 + t * 4.13813679705723846039e-08))));
  const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
#if MPCEKF_PL_BRANCHFREE
  const double v = ldexp(y, (int)k);
  return nan ? x0 : big ? __builtin_inf() : small ? 0.0 : v;
#else
  return ldexp(y, (int)k);
#endif
}

// Electrode tables (include/mpcekf.h mpcekf_electrode; host: build_rom).  In LDS: a
// header [Uocp1 [side][nth] | TK [MAXTT] | soc(0,T), soc(1,T) [side][2][MAXTT]], then
// the 2-D tables [EF_*][side][nte][nth].  EF_CDL is last and only the plant blob
// carries it (k_cell / k_bounds never read Cdleff).  A cell's temperature bracket
// (j, g) is found once per step (bracket); a lookup is then the theta interpolation of
// rows j and j + 1 and a + g (b - a), the sequence of oracle/mpcekf_oracle.c tab2/tidx.
// ABI v3 tables (KRom::npoly): the LDS header holds no Uocp1 and no 2-D tables follow
// but the lookup descriptors; the rows are polynomials in KRom::poly, and a function with
// Ea != 0 is multiplied by its Arrhenius factor dexp(Ea/R (1/Tref - 1/T)).
// permuted row q carries the (single-bit) flag G: bit q of that flag's row mask
__device__ __forceinline__ bool rowf(const KRom &r, int q, unsigned G) {
  return (r.fmask[__builtin_ctz(G)] >> q) & 1u;
}

enum { EF_U = 0, EF_DU, EF_K0, EF_RF, EF_CDL, NEF };
__host__ __device__ constexpr int etab_header(int nth) { return 2 * nth + 5 * MAXTT; }
// v3: the 12 lookup descriptors after the soc ends (d = fn * 2 + side, Uocp1 10 + side),
// KDESC doubles each: Ea/R, then int32 pairs (off, istride), (jstride, ro), (mapoff, nu) as
// raw bits (nu = 0: the uniform grid; v4: the function's bucket map at poly + mapoff)
__host__ __device__ constexpr int etab_desc(int hn) { return 2 * hn + 5 * MAXTT; }
struct ETab {
  const double *b;  // LDS base of the tables
  const KRom *r;    // v3: the polynomial table and the Arrhenius energies
  bool pl;          // v3 tables: a constant of the instantiation (etab<PL>), so each kernel
                    // compiles one lookup (the linear kernels are the round-4 code)
  int nth, nte;
  int hn;           // Uocp1 points in the LDS header: nth (v2), 0 (v3)
  int j;            // temperature bracket of this cell-step
  double g;
  double xa;        // v3: 1/Tref - 1/T of this cell-step (T unclamped)
  // v3 device layout (host build_rom): per function and electrode, interval-major with the
  // nte temperature rows of an interval adjacent, [fn][side][nth-1][nte][KPOLY], so the two
  // rows of a bracket are one 96-byte span; a T-invariant function (all rows equal, e.g. an
  // exact Arrhenius one) keeps one row, [nth-1][1][KPOLY]; Uocp1 last.  Where each function's
  // rows are and its Ea/R come from its descriptor in the LDS header (etab_desc): values in
  // VGPRs read at the lookup, so a kernel holds no per-function scalars (the 2 x 5 offsets
  // and energies as kernel arguments cost ~1,100 SGPR-spill reloads in k_cell).  One code
  // path: the rows of interval i at bracket j are at off + j jstride + i istride and + ro
  // (a T-invariant or single-temperature function: jstride = ro = 0, its row blended with
  // itself, a + g (a - a) = a, oracle tab2)
  __device__ __forceinline__ double f(int side, int fn, double th) const {
    if (pl) {
      const double *dp = b + etab_desc(hn) + (fn * 2 + side) * KDESC;
      const double ear = dp[0];
      const long long w0 = __double_as_longlong(dp[1]), w1 = __double_as_longlong(dp[2]);
      const int off = (int)w0, istr = (int)(w0 >> 32), jstr = (int)w1, ro = (int)(w1 >> 32);
      double a, c;
      int nu = 0, moff = 0;
      if (r->nodes) {  // a uniform flag: v3 ROMs never read the map word
        const long long w3 = __double_as_longlong(dp[3]);
        nu = __builtin_amdgcn_readfirstlane((int)(w3 >> 32));
        moff = __builtin_amdgcn_readfirstlane((int)w3);
      }
      if (nu == 0)
        tabp2(r->poly + off + j * jstr, nth, th, istr, a, c, ro);
      else
        tabn2(r->poly + off + j * jstr, r->poly + moff, nu, th, istr, a, c, ro);
      a = a + g * (c - a);
#if MPCEKF_PL_BRANCHFREE
      // every function multiplied by its factor, dexp(+-0) = 1 exactly when Ea = 0 (a * 1 = a:
      // the oracle's unmultiplied value): no branch between neighbouring lookups' loads
      a = a * dexp(ear != 0.0 ? ear * xa : 0.0);
#else
      if (ear != 0.0) a = a * dexp(ear * xa);
#endif
      return a;
    }
    const double *t = b + etab_header(nth) + ((fn * 2 + side) * nte + j) * nth;
    const double a = tabi(t, nth, th);
    if (nte == 1) return a;
    const double c = tabi(t + nth, nth, th);
    return a + g * (c - a);
  }
  __device__ __forceinline__ double u1(int side, double th) const {
    if (pl) {
      const double *dp = b + etab_desc(hn) + (10 + side) * KDESC;
      const long long w0 = __double_as_longlong(dp[1]);
      if (r->nodes) {
        const long long w3 = __double_as_longlong(dp[3]);
        const int nu = __builtin_amdgcn_readfirstlane((int)(w3 >> 32));
        if (nu) {
          double a, c;
          tabn2(r->poly + (int)w0, r->poly + __builtin_amdgcn_readfirstlane((int)w3), nu, th, (int)(w0 >> 32), a, c, 0);
          return a;
        }
      }
      return tabp(r->poly + (int)w0, nth, th, (int)(w0 >> 32));
    }
    return tabi(b + side * nth, nth, th);
  }
  __device__ __forceinline__ double tk(int i) const { return b[2 * hn + i]; }
  __device__ __forceinline__ double send(int side, int one) const {  // soc(one, T) at the bracket
    const double *t = b + 2 * hn + MAXTT + (side * 2 + one) * MAXTT;
    if (nte == 1) return t[0];
    return t[j] + g * (t[j + 1] - t[j]);
  }
  __device__ __forceinline__ void bracket(double T) {
    j = 0;
    g = 0.0;
    xa = pl && r->arr ? 1.0 / r->Tref - 1.0 / T : 0.0;
    if (nte == 1) return;
    const double Tc = fmin(fmax(T, tk(0)), tk(nte - 1));
    int k = 0;
    while (k < nte - 2 && Tc >= tk(k + 1)) ++k;
    j = k;
    g = (Tc - tk(k)) / (tk(k + 1) - tk(k));
  }
  // soc(z,T) = soc0 + z (soc100 - soc0) (iterEKF.m:282-283)
  __device__ __forceinline__ double soc(int side, double z) const {
    const double s0 = send(side, 0), s1 = send(side, 1);
    return s0 + z * (s1 - s0);
  }
};
template <bool PL>
__device__ __forceinline__ ETab etab(const KRom &r, const double *base, double T) {
  ETab e;
  e.b = base;
  e.r = &r;
  e.pl = PL;
  e.nth = r.nth;
  e.nte = r.nte;
  e.hn = PL ? 0 : r.nth;
  e.bracket(T);
  return e;
}

__device__ __forceinline__ void two_nearest(const double *pts, int n, double x, int &i1, int &i2) {
  int b1 = -1, b2 = -1;
  double d1 = 0.0, d2 = 0.0;
  for (int i = 0; i < n; ++i) {
    double d = fabs(x - pts[i]);
    bool better1 = b1 < 0 || (d < d1) || (d1 != d1 && d == d);
    if (better1) {
      b2 = b1; d2 = d1; b1 = i; d1 = d;
      continue;
    }
    bool better2 = b2 < 0 || (d < d2) || (d2 != d2 && d == d);
    if (better2) { b2 = i; d2 = d; }
  }
  i1 = b1;
  i2 = b2 < 0 ? b1 : b2;
}

struct XI {
  double g[4];
  int m[4];
};

// iterEKF.m:219-255
__device__ __forceinline__ void get_xind(int nT, int nZ, const double *Tp, const double *Zp, double Tk, double SOC,
                                         XI &xi) {
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (nZ > 1) {
    int a, b;
    two_nearest(Zp, nZ, SOC, a, b);
    iZu = a; iZl = b;
    if (Zp[iZu] < Zp[iZl]) { iZu = b; iZl = a; }
  }
  if (nT > 1) {
    int a, b;
    two_nearest(Tp, nT, Tk, a, b);
    iTu = a; iTl = b;
    if (Tp[iTu] < Tp[iTl]) { iTu = b; iTl = a; }
  }
  double aZ = 0.0, aT = 0.0;
  if (nZ > 1) aZ = (SOC - Zp[iZl]) / (Zp[iZu] - Zp[iZl]);
  if (nT > 1) aT = (Tk - Tp[iTl]) / (Tp[iTu] - Tp[iTl]);
  xi.g[0] = (1 - aT) * (1 - aZ);
  xi.g[1] = (1 - aT) * aZ;
  xi.g[2] = aT * (1 - aZ);
  xi.g[3] = aT * aZ;
  xi.m[0] = iTl * nZ + iZl;
  xi.m[1] = iTl * nZ + iZu;
  xi.m[2] = iTu * nZ + iZl;
  xi.m[3] = iTu * nZ + iZu;
}

__device__ __forceinline__ void load_x(const double *rec, double x[NX]) {
  const double2 *p = reinterpret_cast<const double2 *>(rec);
  double2 a = p[0], b = p[1];
  x[0] = a.x; x[1] = a.y; x[2] = b.x; x[3] = b.y;
  x[4] = rec[4];
}
__device__ __forceinline__ void load_rec(const double *rec, double x[NX], double S[NPK]) {
  const double2 *p = reinterpret_cast<const double2 *>(rec);
  double v[REC];
#pragma unroll
  for (int i = 0; i < REC / 2; ++i) {
    double2 t = p[i];
    v[2 * i] = t.x;
    v[2 * i + 1] = t.y;
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) x[i] = v[i];
#pragma unroll
  for (int i = 0; i < NPK; ++i) S[i] = v[NX + i];
}
__device__ __forceinline__ void store_rec(double *rec, const double x[NX], const double S[NPK]) {
  double2 *p = reinterpret_cast<double2 *>(rec);
  double v[REC];
#pragma unroll
  for (int i = 0; i < NX; ++i) v[i] = x[i];
#pragma unroll
  for (int i = 0; i < NPK; ++i) v[NX + i] = S[i];
#pragma unroll
  for (int i = 0; i < REC / 2; ++i) p[i] = make_double2(v[2 * i], v[2 * i + 1]);
}
__device__ __forceinline__ void load_S(const double *rec, double S[NPK]) {
  S[0] = rec[NX];
  const double2 *p = reinterpret_cast<const double2 *>(rec + NX + 1);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    double2 t = p[i];
    S[1 + 2 * i] = t.x;
    S[2 + 2 * i] = t.y;
  }
}

// ---------------------------------------------------------------------------
// Cyclic Jacobi on a packed symmetric 5x5 (orc_jacobi), V row-major 5x5.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void jacobi5(double a[NPK], double V[NX * NX]) {
#pragma unroll
  for (int i = 0; i < NX * NX; ++i) V[i] = (i % (NX + 1)) == 0 ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0, dg = 0.0;
#pragma unroll
    for (int p = 0; p < NX; ++p) {
      dg = dg + a[pk(p, p)] * a[pk(p, p)];
#pragma unroll
      for (int q = p + 1; q < NX; ++q) off = off + a[pk(p, q)] * a[pk(p, q)];
    }
    if (!(off > 1e-36 * dg)) break;
#pragma unroll
    for (int p = 0; p < NX - 1; ++p) {
#pragma unroll
      for (int q = p + 1; q < NX; ++q) {
        double apq = a[pk(p, q)];
        if (apq != 0.0) {
          double theta = (a[pk(q, q)] - a[pk(p, p)]) / (2.0 * apq);
          double t;
          if (fabs(theta) > 1e150) {
            t = 0.5 / theta;
          } else {
            t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
            if (theta < 0) t = -t;
          }
          double c = 1.0 / sqrt(t * t + 1.0), s = t * c, tau = s / (1.0 + c);
          a[pk(p, p)] = a[pk(p, p)] - t * apq;
          a[pk(q, q)] = a[pk(q, q)] + t * apq;
          a[pk(p, q)] = 0.0;
#pragma unroll
          for (int r = 0; r < NX; ++r) {
            if (r == p || r == q) continue;
            double g = a[pk(r, p)], h = a[pk(r, q)];
            a[pk(r, p)] = g - s * (h + g * tau);
            a[pk(r, q)] = h + s * (g - h * tau);
          }
#pragma unroll
          for (int r = 0; r < NX; ++r) {
            double g = V[r * NX + p], h = V[r * NX + q];
            V[r * NX + p] = g - s * (h + g * tau);
            V[r * NX + q] = h + s * (g - h * tau);
          }
        }
      }
    }
  }
}

// Positive definiteness of a packed symmetric 5x5 by LDL' pivots (orc_is_pd, same order).
// sc: a = sc * the given array (1.0: a itself), applied where an entry is read.
__device__ __forceinline__ bool is_pd5(const double a[NPK], double sc = 1.0) {
  double l[NX][NX], d[NX];
  bool pd = true;
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double s = a[pk(j, j)] * sc;
#pragma unroll
    for (int k = 0; k < j; ++k) s = __builtin_fma(-(l[j][k] * l[j][k]), d[k], s);
    pd = pd && (s > 0);
    d[j] = s;
    if (j + 1 < NX) {
      const double inv = 1.0 / s;
#pragma unroll
      for (int i = j + 1; i < NX; ++i) {
        double t = a[pk(j, i)] * sc;
#pragma unroll
        for (int k = 0; k < j; ++k) t = __builtin_fma(-(l[i][k] * l[j][k]), d[k], t);
        l[i][j] = t * inv;
      }
    }
  }
  return pd;
}

// The symmetrisation of meas_update_regs when some lane of the wave is not positive
// definite: HH = V|Lambda|V' by Jacobi (out of line: rare, and its registers would
// otherwise weigh on every caller).
template <bool INL>
__device__ __forceinline__ void meas_polar(const double Ps[NPK], double a[NPK], double S[NPK], bool pd, bool bump) {
  double H[NPK];
#pragma unroll
  for (int i = 0; i < NPK; ++i) H[i] = a[i];
  double V[NX * NX];
  jacobi5(a, V);
  double w[NX];
#pragma unroll
  for (int k = 0; k < NX; ++k) w[k] = fabs(a[pk(k, k)]);
#pragma unroll
  for (int r = 0; r < NX; ++r)
#pragma unroll
    for (int c = r; c < NX; ++c) {
      double hrc = 0.0, hcr = 0.0;
#pragma unroll
      for (int k = 0; k < NX; ++k) {
        hrc = hrc + (V[r * NX + k] * w[k]) * V[c * NX + k];
        hcr = hcr + (V[c * NX + k] * w[k]) * V[r * NX + k];
      }
      if (pd) { hrc = H[pk(r, c)]; hcr = H[pk(r, c)]; }
      double v = ((Ps[pk(r, c)] + hrc) + hcr) / 4.0;
      if (bump) v = v * 2.0;
      S[pk(r, c)] = v;
    }
}

__device__ __noinline__ void meas_polar_slow(const double Ps[NPK], double a[NPK], double S[NPK], bool pd,
                                             bool bump) {
  meas_polar<false>(Ps, a, S, pd, bump);
}

// iterEKF.m:137-153 on one corner record (orc_meas_cov + state update).
// P = Sigma - (L*St)*L' is only ever used as P + P', so only that sum is kept.
template <bool OUTLINE = false>  // OUTLINE: the Jacobi branch as a call (k_ekf4's 128/256-VGPR budget)
__device__ __forceinline__ void meas_update_regs(double x[NX], double S[NPK], const double L[NX], double St,
                                                 double res) {
#pragma unroll
  for (int k = 0; k < NX; ++k) x[k] = __builtin_fma(L[k], res, x[k]);
  double LS[NX];
#pragma unroll
  for (int r = 0; r < NX; ++r) LS[r] = L[r] * St;
  double Ps[NPK];
#pragma unroll
  for (int r = 0; r < NX; ++r)
#pragma unroll
    for (int c = r; c < NX; ++c) {
      double prc = __builtin_fma(-LS[r], L[c], S[pk(r, c)]);
      double pcr = __builtin_fma(-LS[c], L[r], S[pk(r, c)]);
      Ps[pk(r, c)] = prc + pcr;
    }
  // a = (P + P')/2 = Ps * 0.5: the same operation on the same sum, formed where it is
  // used (not held: an array of 15 doubles less at the kernel's register peak)
  const bool bump = res * res > 9 * St;
  // HH = VV*SS*VV' (iterEKF.m:145-146) is the polar factor of the symmetric part a:
  // a itself when a is positive definite (the usual case), else V|Lambda|V' (Jacobi).
  // The decomposition runs only if some lane of the wave needs it.
  const bool pd = is_pd5(Ps, 0.5);
  if (__all(pd)) {
#pragma unroll
    for (int i = 0; i < NPK; ++i) {
      const double a = Ps[i] * 0.5;
      double v = ((Ps[i] + a) + a) / 4.0;
      if (bump) v = v * 2.0;
      S[i] = v;
    }
  } else {
    double a[NPK];
#pragma unroll
    for (int i = 0; i < NPK; ++i) a[i] = Ps[i] * 0.5;
    if constexpr (OUTLINE) meas_polar_slow(Ps, a, S, pd, bump);
    else meas_polar<true>(Ps, a, S, pd, bump);
  }
}

__device__ __forceinline__ void meas_update(double *rec, const double L[NX], double St, double res) {
  double x[NX], S[NPK];
  load_rec(rec, x, S);
  meas_update_regs(x, S, L, St, res);
  store_rec(rec, x, S);
}

// ---------------------------------------------------------------------------
// Per-lane context for one cell
// ---------------------------------------------------------------------------
struct CellCtx {
  const double *L;   // LDS: model blob base
  const double *Tp, *Zp;  // LDS set-points
  double *erec;      // this cell's EKF records in HBM
  int stride;
  double T;          // iterEKF's Tk in K (iterEKF.m:62-66)
  ETab et;           // electrode tables, bracketed at T
};

// getVariables (iterEKF.m:259-417).  Z is the permuted output vector.
// QUAD: a lane quad per cell (k_ekf4): this lane's corner is qj with state xr[0]; the
// corner sums Z = fma(z_j, g_j, Z), j = 0..3 in order, take z_j from lane j by DPP.
// k0 and Rf of one getVariables call at its SOCnAvg / SOCpAvg (after its clamps): getChatV
// (the same x0), getChatZ's scalars and EKFmatsHandler (the same x0 after the update) read
// k0 / Rf at the unclamped averages, which are these whenever no clamp fired -- the same
// lookup, so the same bits; they reuse the values then (fewer table reads, notably of
// the v3 polynomials) and look up otherwise
struct KR {
  double T, thn, thp, k0n, k0p, rfn, rfp;  // T: the lookups' temperature (EKFmatsHandler brackets its own)
};
__device__ __forceinline__ bool kr_hit(const KR *kr, double T, double thn, double thp) {
  return kr && kr->T == T && kr->thn == thn && kr->thp == thp;
}
template <int NZ, bool QUAD = false>
__device__ __forceinline__ double get_vars(const KRom &r, const CellCtx &cc, const XI &xi, double ik, double x0,
                                           double SOC0, int &warn, int &st, double Z[NZ], double &Zsoc,
                                           const double (*xr)[NX] = nullptr, int qj = 0, KR *kr = nullptr) {
  double xSOC = SOC0 - x0 * (r.Ts / (3600 * r.Q));
  double SOCnAvg = cc.et.soc(0, xSOC);
  double SOCpAvg = cc.et.soc(1, xSOC);
  if (SOCnAvg < 0) { warn++; SOCnAvg = 1e-6; }
  if (SOCnAvg > 1) { warn++; SOCnAvg = 1 - 1e-6; }
  if (SOCpAvg < 0) { warn++; SOCpAvg = 1e-6; }
  if (SOCpAvg > 0.998) { warn++; SOCpAvg = 0.998; }
#pragma unroll
  for (int q = 0; q < NZ; ++q) Z[q] = 0.0;
  if constexpr (QUAD) {
    const double *Cm = cc.L + xi.m[qj] * cc.stride;
    const double *Dm = Cm + NZ * NX;
    double cr[NX + 1];
#pragma unroll
    for (int k = 0; k < NX; ++k) cr[k] = Cm[k];
    cr[NX] = Dm[0];
#pragma unroll
    for (int q = 0; q < NZ; ++q) {
      double cn[NX + 1];
      if (q + 1 < NZ) {
#pragma unroll
        for (int k = 0; k < NX; ++k) cn[k] = Cm[(q + 1) * NX + k];
        cn[NX] = Dm[q + 1];
      }
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < NX; ++k) acc = __builtin_fma(cr[k], xr[0][k], acc);
      const double zj = __builtin_fma(cr[NX], ik, acc);
      double zz = __builtin_fma(qbc<0>(zj), xi.g[0], 0.0);
      zz = __builtin_fma(qbc<1>(zj), xi.g[1], zz);
      zz = __builtin_fma(qbc<2>(zj), xi.g[2], zz);
      Z[q] = __builtin_fma(qbc<3>(zj), xi.g[3], zz);
      launder(Z[q]);  // rows in order: the next row's operands are the only ones in flight
      if (q + 1 < NZ) {
#pragma unroll
        for (int k = 0; k <= NX; ++k) cr[k] = cn[k];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < (QUAD ? 0 : 4); ++j) {
    double x[NX];
    if (xr) {
#pragma unroll
      for (int k = 0; k < NX; ++k) x[k] = xr[j][k];
    } else {
      load_x(cc.erec + (size_t)xi.m[j] * REC, x);
    }
    const double *Cm = cc.L + xi.m[j] * cc.stride;
    const double *Dm = Cm + NZ * NX;
    double g = xi.g[j];
    // row q+1's C and D are read while row q computes (LDS latency off the chain)
    double cr[NX + 1];
#pragma unroll
    for (int k = 0; k < NX; ++k) cr[k] = Cm[k];
    cr[NX] = Dm[0];
#pragma unroll
    for (int q = 0; q < NZ; ++q) {
      double cn[NX + 1];
      if (q + 1 < NZ) {
#pragma unroll
        for (int k = 0; k < NX; ++k) cn[k] = Cm[(q + 1) * NX + k];
        cn[NX] = Dm[q + 1];
      }
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < NX; ++k) acc = __builtin_fma(cr[k], x[k], acc);
      const double zj = __builtin_fma(cr[NX], ik, acc);
      Z[q] = __builtin_fma(zj, g, Z[q]);
      launder(Z[q]);
      if (q + 1 < NZ) {
#pragma unroll
        for (int k = 0; k <= NX; ++k) cr[k] = cn[k];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_sched_barrier(0);
  double If0 = Z[R_IF0], If3 = Z[R_IF3];
  bool any = false;
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_NTH)) { Z[q] = Z[q] + SOCnAvg; any |= Z[q] < 0; }
  if (any) {
    warn++;
#pragma unroll
    for (int q = 0; q < NZ; ++q)
      if ((rowf(r, q, G_NTH)) && Z[q] < 0) Z[q] = 1e-6;
  }
  any = false;
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_NTH)) any |= Z[q] > 1;
  if (any) {
    warn++;
#pragma unroll
    for (int q = 0; q < NZ; ++q)
      if ((rowf(r, q, G_NTH)) && Z[q] > 1) Z[q] = 1 - 1e-6;
  }
  any = false;
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_PTH)) { Z[q] = Z[q] + SOCpAvg; any |= Z[q] < 0; }
  if (any) {
    warn++;
#pragma unroll
    for (int q = 0; q < NZ; ++q)
      if ((rowf(r, q, G_PTH)) && Z[q] < 0) Z[q] = 1e-6;
  }
  any = false;
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_PTH)) any |= Z[q] > 0.998;
  if (any) {
    warn++;
#pragma unroll
    for (int q = 0; q < NZ; ++q)
      if ((rowf(r, q, G_PTH)) && Z[q] > 0.998) Z[q] = 0.998;
  }
  double Un = cc.et.f(0, EF_U, SOCnAvg), Up = cc.et.f(1, EF_U, SOCpAvg);
#pragma unroll
  for (int q = 0; q < NZ; ++q) {
    if (rowf(r, q, G_NPHISE)) Z[q] = Z[q] + Un;
    if (rowf(r, q, G_PPHISE)) Z[q] = Z[q] + Up;
  }
  double PhieTilde3 = Z[R_PHIE];
  double Phise0 = Z[R_PHISE0];
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_PHIE)) {
      if (rowf(r, q, G_PHIE0)) Z[q] = 0 - Phise0;
      else Z[q] = Z[q] - Phise0;
    }
  any = false;
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_THETAE)) { Z[q] = Z[q] + 1; any |= Z[q] < 0; }
  if (any) {  // iterEKF.m:384-389 would raise a MATLAB error
    warn++;
    st |= ST_ERROR | ST_THETAE_NEG;
    return __builtin_nan("");
  }
  double k0n = cc.et.f(0, EF_K0, SOCnAvg), k0p = cc.et.f(1, EF_K0, SOCpAvg);  // iterEKF.m:392-393
  double i0n = k0n * sqrt(Z[R_TE1] * (1 - Z[R_TH0]) * Z[R_TH0]);
  double i0p = k0p * sqrt(Z[R_TEE] * (1 - Z[R_TH3]) * Z[R_TH3]);
  double negEta0 = 2 * r.R * cc.T / r.F * dasinh(If0 / (2 * i0n));
  double posEta3 = 2 * r.R * cc.T / r.F * dasinh(If3 / (2 * i0p));
  double Uocpn0 = cc.et.f(0, EF_U, Z[R_TH0]), Uocpp3 = cc.et.f(1, EF_U, Z[R_TH3]);
  double Rfn = cc.et.f(0, EF_RF, SOCnAvg), Rfp = cc.et.f(1, EF_RF, SOCpAvg);  // iterEKF.m:406-407
  if (kr) *kr = KR{cc.T, SOCnAvg, SOCpAvg, k0n, k0p, Rfn, Rfp};
  double V = posEta3 - negEta0 + PhieTilde3 + Uocpp3 - Uocpn0 + (Rfp * Z[R_IFDL3] - Rfn * Z[R_IFDL0]);
#pragma unroll
  for (int q = 0; q < NZ; ++q)
    if (rowf(r, q, G_PPHIS)) Z[q] = Z[q] + V;
  Zsoc = SOC0 - x0 * (r.Ts / (3600 * r.Q));
  return V;
}

// getChatV (iterEKF.m:421-519) pieces.  Cell scalars of the voltage Jacobian.
struct ChatK {
  double Rfn, Rfp, Rctn, Rctp, dUn0, dUp3, dn, dp;
};
// xSOC = SOC0 - x0 Ts/(3600 Q) with the x0 of the call: Rf and k0 at the unclamped
// soc(xSOC, Tk) (iterEKF.m:437-442,463-464)
__device__ __forceinline__ ChatK chat_k(const KRom &r, const CellCtx &cc, double xSOC, double zTE1, double zTH0,
                                        double zTEE, double zTH3, const KR *kr = nullptr) {
  ChatK k;
  const double SOCnAvg = cc.et.soc(0, xSOC), SOCpAvg = cc.et.soc(1, xSOC);
  double k0n, k0p;
  if (kr_hit(kr, cc.T, SOCnAvg, SOCpAvg)) {
    k.Rfn = kr->rfn;
    k.Rfp = kr->rfp;
    k0n = kr->k0n;
    k0p = kr->k0p;
  } else {
    k.Rfn = cc.et.f(0, EF_RF, SOCnAvg);
    k.Rfp = cc.et.f(1, EF_RF, SOCpAvg);
    k0n = cc.et.f(0, EF_K0, SOCnAvg);
    k0p = cc.et.f(1, EF_K0, SOCpAvg);
  }
  double i0n = k0n * sqrt(zTE1 * (1 - zTH0) * zTH0);
  double i0p = k0p * sqrt(zTEE * (1 - zTH3) * zTH3);
  k.Rctn = r.R * cc.T / (r.F * i0n);
  k.Rctp = r.R * cc.T / (r.F * i0p);
  k.dUn0 = cc.et.f(0, EF_DU, zTH0);
  k.dUp3 = cc.et.f(1, EF_DU, zTH3);
  k.dn = cc.et.soc(0, 1) - cc.et.soc(0, 0);  // soc(1,Tk) - soc(0,Tk) (iterEKF.m:497-500)
  k.dp = cc.et.soc(1, 1) - cc.et.soc(1, 0);
  return k;
}
// The row of one corner (model blob Cm, interpolation weight g).
__device__ __forceinline__ void chat_row(const KRom &r, const ChatK &K, const double *Cm, double g, double Chat[NX]) {
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    double v = K.Rfp * (g * Cm[R_IFDL3 * NX + k]) - K.Rfn * (g * Cm[R_IFDL0 * NX + k]);
    v = v + K.Rctp * (g * Cm[R_IF3 * NX + k]) - K.Rctn * (g * Cm[R_IF0 * NX + k]);
    v = v + g * Cm[R_PHIE * NX + k];
    v = v + (K.dUp3 * (g * Cm[R_TH3 * NX + k]) - K.dUn0 * (g * Cm[R_TH0 * NX + k]));
    Chat[k] = v;
  }
}
__device__ __forceinline__ double chat0(const KRom &r, const ChatK &K) {
  double res0n = -K.dUn0 * r.Ts * K.dn / (3600 * r.Q);
  double res0p = -K.dUp3 * r.Ts * K.dp / (3600 * r.Q);
  return res0p - res0n;
}
// Voltage Jacobian rows of the 4 corners.
template <int NZ>
__device__ __forceinline__ void get_chatv(const KRom &r, const CellCtx &cc, const XI &xi, double xSOC, double zTE1,
                                          double zTH0, double zTEE, double zTH3, double Chat[4][NX], double &Chat0,
                                          const KR *kr = nullptr) {
  const ChatK K = chat_k(r, cc, xSOC, zTE1, zTH0, zTEE, zTH3, kr);
#pragma unroll
  for (int j = 0; j < 4; ++j) chat_row(r, K, cc.L + xi.m[j] * cc.stride, xi.g[j], Chat[j]);
  Chat0 = chat0(r, K);
}

// getChatZ's scalars at the updated state (iterEKF.m:190, 543, 562-580): for k_bounds
struct BoundK {
  ChatK K;
  double C0, r0n, r0p, dUn, dUp;
};
__device__ __forceinline__ BoundK bound_k(const KRom &r, const CellCtx &cc, double xSOC, double zTE1, double zTH0,
                                          double zTEE, double zTH3, const KR *kr = nullptr) {
  BoundK b;
  b.K = chat_k(r, cc, xSOC, zTE1, zTH0, zTEE, zTH3, kr);
  b.C0 = chat0(r, b.K);
  b.r0n = -r.Ts * b.K.dn / (3600 * r.Q);  // iterEKF.m:562-565
  b.r0p = -r.Ts * b.K.dp / (3600 * r.Q);
  b.dUn = cc.et.f(0, EF_DU, cc.et.soc(0, xSOC));  // iterEKF.m:576-580
  b.dUp = cc.et.f(1, EF_DU, cc.et.soc(1, xSOC));
  return b;
}
__device__ __forceinline__ double bound_field(const BoundK &b, int i) {  // BD_K + i, i < 11
  switch (i) {
    case 0: return b.K.Rfn;
    case 1: return b.K.Rfp;
    case 2: return b.K.Rctn;
    case 3: return b.K.Rctp;
    case 4: return b.K.dUn0;
    case 5: return b.K.dUp3;
    case 6: return b.C0;
    case 7: return b.r0n;
    case 8: return b.r0p;
    case 9: return b.dUn;
    default: return b.dUp;
  }
}

// MPC pieces (predMat.m, constraintsMPC.m, iterMPC.m) live in mpcekf_mpc.hpp,
// templated on the horizons; this file instantiates them for NP x NC.
using Cons = ConsT<NP, NC>;
using MpcSetup = MpcSetupT<NP, NC>;

// EKFmatsHandler.m:26-114.  zTE1.. are the role rows of zk, Zsoc = zk(end).
// EKFmatsHandler.m:26-31: the corner of largest weight, first of equals; max()
// skips NaN weights.
// The running maximum and its model index are carried in registers: xi.g[imax] / xi.m[imax]
// with a run-time imax would keep the whole XI in scratch.
__device__ __forceinline__ int corner_max(const XI &xi, int *mmax = nullptr) {
  int imax = 0, m = xi.m[0];
  double gm = xi.g[0];
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    const double gj = xi.g[j];
    int mj = xi.m[j];
    asm("" : "+v"(mj));  // a value: a select of two loads would be folded into one indexed load
    if (gj > gm || (gm != gm && gj == gj)) {
      imax = j;
      gm = gj;
      m = mj;
    }
  }
  if (mmax) *mmax = m;
  return imax;
}

// xm (use_xm): that corner's xhat when the caller holds it in registers (k_cell's fused
// step), else read from its record
template <int NZ>
__device__ __forceinline__ void mats_handler(const KRom &r, const CellCtx &cc, const XI &xi, const double *zr,
                                             double Zsoc, double TK, Lin &L, double xend, const double (&xm)[NX],
                                             bool use_xm, const KR *kr = nullptr) {
  int m;
  (void)corner_max(xi, &m);
  const double *Cm = cc.L + m * cc.stride;
  const double *Dm = Cm + NZ * NX;
  const double *am = Dm + NZ;
  double x[NX];
  if (use_xm) {
#pragma unroll
    for (int k = 0; k < NX; ++k) x[k] = xm[k];
  } else {
    load_x(cc.erec + (size_t)m * REC, x);
  }
#pragma unroll
  for (int k = 0; k < NX; ++k) { L.xhat[k] = x[k]; L.a[k] = am[k]; }
  L.xhat[NX] = xend;  // ekfData.xhat(end) (EKFmatsHandler.m:33): 0 in 'OB', the MB integrator
  L.a[NX] = 1.0;
  double rr = -r.Ts / (3600 * r.Q);
#pragma unroll
  for (int k = 0; k < 6; ++k) L.Csoc[k] = 0.0;
  L.Csoc[NX] = rr;
  L.Dsoc = 0.0;
  ETab et = cc.et;
  et.bracket(TK);  // EKFmatsHandler.m:53: TK = Tk + 273.15
  double SOCnAvg = et.soc(0, Zsoc), SOCpAvg = et.soc(1, Zsoc);  // EKFmatsHandler.m:57-58
  double k0n, k0p, Rfn, Rfp;  // EKFmatsHandler.m:60-61,68-69 (the second getVariables' when its averages)
  if (kr_hit(kr, TK, SOCnAvg, SOCpAvg)) {
    k0n = kr->k0n;
    k0p = kr->k0p;
    Rfn = kr->rfn;
    Rfp = kr->rfp;
  } else {
    k0n = et.f(0, EF_K0, SOCnAvg);
    k0p = et.f(1, EF_K0, SOCpAvg);
    Rfn = et.f(0, EF_RF, SOCnAvg);
    Rfp = et.f(1, EF_RF, SOCpAvg);
  }
  double i0n = k0n * sqrt(zr[R_TE1] * (1 - zr[R_TH0]) * zr[R_TH0]);
  double i0p = k0p * sqrt(zr[R_TEE] * (1 - zr[R_TH3]) * zr[R_TH3]);
#pragma unroll
  for (int k = 0; k < NX; ++k)
    L.Cv[k] = Rfp * Cm[R_IFDL3 * NX + k] - Rfn * Cm[R_IFDL0 * NX + k] + Cm[R_PHIE * NX + k];
  L.Cv[NX] = 0.0;
  L.Dv = Rfp * Dm[R_IFDL3] - Rfn * Dm[R_IFDL0] + Dm[R_PHIE];
  double Upos = et.f(1, EF_U, zr[R_TH3]), Uneg = et.f(0, EF_U, zr[R_TH0]);
  double negEta0 = 2 * r.R * TK / r.F * dasinh(zr[R_IF0] / (2 * i0n));
  double posEta3 = 2 * r.R * TK / r.F * dasinh(zr[R_IF3] / (2 * i0p));
  double b_phi = 0.01 * 0;
  L.bv = (Upos - Uneg) + (posEta3 - negEta0) + b_phi;
  L.bphi = et.u1(0, SOCnAvg);  // one-argument Uocp (EKFmatsHandler.m:96)
#pragma unroll
  for (int k = 0; k < NX; ++k) L.Cphi[k] = Cm[R_NPHISE2 * NX + k];
  L.Cphi[NX] = 0.0;
  L.Dphi = Dm[R_NPHISE2];
}

// hildreth.m:17-46.  H = M*(E\M') is re-formed entry by entry in the exact
// summation order of the dense product (orc_hildreth), never stored.
template <class MV>
__device__ __forceinline__ int hildreth_core(const MV &Mf, const double E[NC][NC], const double F[NC],
                                             const double gam[NCON], double lam[NCON], int maxIter, double tol,
                                             double DU[NC]) {
  double R[NC][NC];
  bool ok = chol_n<NC>(E, R);
  double X[NCON][NC];
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    double b[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) b[k] = Mf(i, k);
    mldiv_spd<NC>(E, R, ok, b, X[i]);
  }
  double y[NC];
  mldiv_spd<NC>(E, R, ok, F, y);
  double K[NCON];
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) s = s + Mf(i, k) * y[k];
    K[i] = s + gam[i];
  }
  bool fin = true;
#pragma unroll
  for (int i = 0; i < NCON; ++i)
#pragma unroll
    for (int k = 0; k < NC; ++k) fin = fin && isfinite(X[i][k]) && isfinite(Mf(i, k));
  // orc_hildreth's defined evaluation: rank-Nc form with v = X*lambda when X and M are
  // finite, else the dense H(i,:)*lambda as 4 interleaved partial sums
  auto xv = [&](double v[NC]) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < NCON; ++j) a = __builtin_fma(X[j][k], lam[j], a);
      v[k] = a;
    }
  };
  int it;
  for (it = 1; it <= maxIter; ++it) {
#pragma unroll
    for (int i = 0; i < NCON; ++i)
#pragma unroll
      for (int k = 0; k < NC; ++k) launder(X[i][k]);
    bool conv = true;
    double v[NC];
    if (fin) xv(v);
#pragma unroll
    for (int i = 0; i < NCON; ++i) {
      double hii = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) hii = hii + Mf(i, k) * X[i][k];
      double s = 0.0, nl, d;
      if (fin) {
        double t = K[i];
#pragma unroll
        for (int k = 0; k < NC; ++k) t = __builtin_fma(Mf(i, k), v[k], t);
        d = hild_step(t, hii, 1.0 / hii, lam[i], nl);
      } else {
        double p4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NCON; ++j) {
          double h = 0.0;
#pragma unroll
          for (int k = 0; k < NC; ++k) h = h + Mf(i, k) * X[j][k];
          p4[j & 3] = p4[j & 3] + h * lam[j];
        }
        s = (p4[0] + p4[1]) + (p4[2] + p4[3]);
        const double w = -((K[i] + s) - hii * lam[i]) / hii;
        nl = w > 0 ? w : 0.0;
        d = nl - lam[i];
      }
      if (!(fabs(d) < tol)) conv = false;
      lam[i] = nl;
      if (fin) {
        if (isfinite(d)) {
#pragma unroll
          for (int k = 0; k < NC; ++k) v[k] = __builtin_fma(X[i][k], d, v[k]);
        } else {
          xv(v);
        }
      }
    }
    if (conv) break;
  }
  if (it > maxIter) it = maxIter;
  double rhs[NC], mE[NC][NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NCON; ++i) s = s + Mf(i, k) * lam[i];
    rhs[k] = F[k] + s;
  }
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) mE[a][b] = -E[a][b];
  lu_solve_n<NC>(mE, rhs, DU);
  return it;
}

struct ConsM {
  const Cons &C;
  __device__ __forceinline__ double operator()(int i, int k) const { return mval(C, i, k); }
};
struct DenseM {
  const double (&M)[NCON][NC];
  __device__ __forceinline__ double operator()(int i, int k) const { return M[i][k]; }
};

// Hildreth problem record handed from k_cell to k_hild, SoA [field][cell].
enum { PB_E = 0, PB_F = PB_E + NC * NC, PB_HV = PB_F + NC, PB_HE = PB_HV + NP, PB_HS = PB_HE + NP,
       PB_GAM = PB_HS + NP, PB_ERR = PB_GAM + NCON, PB_RU = PB_ERR + NP, PB_UK1 = PB_RU + 1, PB_N = PB_UK1 + 1 };

static_assert(PB_N == PROB_DOUBLES, "problem record size");

// hildreth.m:17-46.  H(i,:)*lambda is summed in orc_hildreth's defined order: four
// interleaved partial sums p_q (terms j = q mod 4, each from +0 in ascending j),
// combined as (p0 + p1) + (p2 + p3).  None of these sums can be -0.
//
// X = E\M' is kept for the 15 Toeplitz rows plus three solves for the constant
// current rows: X(-b) = -X(b) exactly under round-to-nearest; the sign of a
// zero in those X entries cannot reach the sweep (it only feeds products added to
// sums that are never -0, and their diagonal H_ii = E^-1_00 > 0).
struct XS {
  double a[NC], b[NC], c[NC];        // E\[1;0], E\[1;1], E\[0;1]
  double t[3 * NP][NC];              // E\M(i,:)' for the V / eta / SOC rows
};
__device__ __forceinline__ double xval(const XS &X, int j, int k) {
  switch (j) {  // rows of [Cu; -Cu; I; -I] for NC == 2
    case 0: return X.a[k];
    case 1: return X.b[k];
    case 2: return -X.a[k];
    case 3: return -X.b[k];
    case 4: return X.a[k];
    case 5: return X.c[k];
    case 6: return -X.a[k];
    case 7: return -X.c[k];
    default: return X.t[j - 4 * NC][k];
  }
}

// X = E\M' in compressed form (hildreth.m:25); fin = every X and M entry finite.
__device__ __forceinline__ void hild_x(const Cons &Cn, const double E[NC][NC], XS &Xs, bool &fin) {
  ConsM Mf{Cn};
  double R[NC][NC];
  bool ok = chol_n<NC>(E, R);
  {
    double b1[NC] = {1.0, 0.0}, b2[NC] = {1.0, 1.0}, b3[NC] = {0.0, 1.0};
    mldiv_spd<NC>(E, R, ok, b1, Xs.a);
    mldiv_spd<NC>(E, R, ok, b2, Xs.b);
    mldiv_spd<NC>(E, R, ok, b3, Xs.c);
  }
#pragma unroll
  for (int i = 4 * NC; i < NCON; ++i) {
    double b[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) b[k] = Mf(i, k);
    mldiv_spd<NC>(E, R, ok, b, Xs.t[i - 4 * NC]);
  }
  fin = true;
#pragma unroll
  for (int j = 0; j < NCON; ++j)
    fin = fin && isfinite(xval(Xs, j, 0)) && isfinite(xval(Xs, j, 1)) && isfinite(Mf(j, 0)) && isfinite(Mf(j, 1));
}

// Per-lane LDS of the rank-2 sweeps: the 18 distinct X(:,i) (rows 0-7 of
// [Cu; -Cu; I; -I] are +-a, +-b, +-c) and the 18 distinct (H_ii, 1/H_ii) pairs (H_ii of
// a negated row is bit-identical: (-1)(-x) = x, and its 0 * (-x) term only meets
// a nonzero sum or +0).  Layout [slot][64 lanes] double2: every read is one
// conflict-free ds_read_b128 per wave.  1/H_ii is the correctly rounded reciprocal of hild_step.
constexpr int HS_X = 3 + 3 * NP, HS_SLOTS = 2 * HS_X;
constexpr int HILD_LDS_PER_WAVE = HS_SLOTS * 64 * 16;  // bytes
__device__ __forceinline__ constexpr int hslot(int i) {
  return i >= 8 ? 3 + (i - 8) : (i == 1 || i == 3) ? 1 : (i == 5 || i == 7) ? 2 : 0;
}
__device__ __forceinline__ constexpr bool hneg(int i) { return i == 2 || i == 3 || i == 6 || i == 7; }
// The first row of each Toeplitz block is (H(0), 0): all zero when H(0) = 0, as for the
// SOC block (predMat: G(1,1) = +0), so its H_ii may be 0; 1/H_ii is then +-inf and hild_step's
// product gives x / +-0's inf / NaN by IEEE without a select.
__device__ __forceinline__ double2 hx(const double2 *hl, int i) {  // X(:,i)
  const double2 x = hl[hslot(i) * 64];
  return hneg(i) ? make_double2(-x.x, -x.y) : x;
}
__device__ __forceinline__ double2 hh(const double2 *hl, int i) {  // (H_ii, 1/H_ii)
  return hl[(HS_X + hslot(i)) * 64];
}
__device__ __forceinline__ double2 *hild_lane_lds(double2 *base) {  // blocks of 256 threads
  return base + (threadIdx.x >> 6) * (HS_SLOTS * 64) + (threadIdx.x & 63);
}
// Fills the lane's slots; returns whether every H_ii is in hild_step's reciprocal domain
// (hild_rok: 0 or [2^-1020, 2^1020]), where a row is min(t (1/H_ii), lambda_i).
__device__ __forceinline__ bool hild_stage(const Cons &Cn, const XS &Xs, double2 *hl) {
  ConsM Mf{Cn};
  bool yok = true;
#pragma unroll
  for (int sl = 0; sl < HS_X; ++sl) {
    const int i = sl == 0 ? 0 : sl == 1 ? 1 : sl == 2 ? 5 : 8 + (sl - 3);  // representative row
    const double x0 = xval(Xs, i, 0), x1 = xval(Xs, i, 1);
    const double hii = (0.0 + Mf(i, 0) * x0) + Mf(i, 1) * x1;  // orc_hildreth's H(i,i)
    yok = yok && hild_rok(hii);
    hl[sl * 64] = make_double2(x0, x1);
    hl[(HS_X + sl) * 64] = make_double2(hii, 1.0 / hii);  // the oracle's 1.0 / hii (IEEE)
  }
  return yok;
}
__device__ __forceinline__ void hild_unstage(const double2 *hl, XS &Xs) {
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    Xs.a[k] = k ? hl[0].y : hl[0].x;
    Xs.b[k] = k ? hl[64].y : hl[64].x;
    Xs.c[k] = k ? hl[128].y : hl[128].x;
  }
#pragma unroll
  for (int i = 0; i < 3 * NP; ++i) {
    const double2 x = hl[(3 + i) * 64];
    Xs.t[i][0] = x.x;
    Xs.t[i][1] = x.y;
  }
}

// One rank-2 sweep (orc_hildreth, finite X and M): v = X*lambda from +0 at the sweep
// start (fma, ascending j), t_i = fma(M_i1, v1, fma(M_i0, v0, K_i)),
// m = min(t_i (1/H_ii), lambda_i), d = -m, lambda_i -= m (hild_step with every H_ii in its
// domain and lambda finite), v += X(:,i) * d by fma.  A row's dependent chain is t (2 fma) ->
// q -> min -> v: 5 operations (10 with round 5's division); the new lambda_i is beside it and
// can take lambda_i's register (no rotation of the 23 lambdas at the sweep's end).
// The fast form: straight line, no frozen lanes (the caller keeps a converged lane's
// lambda aside).  It reports max |d| (the reference's inf-norm test, hildreth.m:39) and
// whether v ended finite (false once any d was not finite: inf and NaN stay in v; every
// lambda was finite until then, so each row was hild_step's reciprocal form).
// The constant rows 0-7 ([Cu; -Cu; I; -I]) use 3 of the 18 slots (X: +-a, +-b, +-c; their
// (H_ii, 1/H_ii)): those 6 pairs are held in registers (xr3 / hr3, read back from the
// lane's LDS slots once per solve), so a sweep reads LDS for the 15 Toeplitz rows only.
// At 4 waves per CU in the maxIter window the two ds_read_b128 per row were as long as
// the row's dependent chain.
constexpr int HILD_REG_ROWS = MPCEKF_HILD_REGROWS ? 4 * NC : 0;
__device__ __forceinline__ double2 hx_r(const double2 *hl, const double2 xr3[3], int i) {
  if (i < HILD_REG_ROWS) {
    const double2 x = xr3[hslot(i)];
    return hneg(i) ? make_double2(-x.x, -x.y) : x;
  }
  return hx(hl, i);
}
__device__ __forceinline__ double2 hh_r(const double2 *hl, const double2 hr3[3], int i) {
  return i < HILD_REG_ROWS ? hr3[hslot(i)] : hh(hl, i);
}
// M(i, k) is a structural zero of constraintsMPC.m's M (a constant of the unrolled row loop)
__device__ __forceinline__ constexpr bool mzero(int i, int k) {
  return i < NC ? k > i
       : i < 2 * NC ? k > i - NC
       : i < 3 * NC ? (i - 2 * NC) != k
       : i < 4 * NC ? (i - 3 * NC) != k
       : i < 4 * NC + NP ? k > i - 4 * NC
       : i < 4 * NC + 2 * NP ? k > i - 4 * NC - NP
                             : k > i - 4 * NC - 2 * NP;
}
// v = X*lambda from +0 in ascending j (the sweep-start v of orc_hildreth)
__device__ __forceinline__ void hild_v(const double2 *hl, const double2 xr3[3], const double L[NCON], double &v0,
                                       double &v1) {
  v0 = 0.0;
  v1 = 0.0;
#pragma unroll
  for (int j = 0; j < NCON; ++j) {
    const double2 x = hx_r(hl, xr3, j);
    v0 = __builtin_fma(x.x, L[j], v0);
    v1 = __builtin_fma(x.y, L[j], v1);
  }
}
// (v0, v1): this sweep's start v in, the next sweep's out.  The next sweep's v is summed
// row by row from lambda_i's final value of this sweep (row i is the last to change it),
// the same fmas on the same operands in the same order as hild_v after the sweep, with the
// X(:,i) the row already read (MPCEKF_HILD_NEXTV; 0: hild_v at every sweep start).
__device__ __forceinline__ void sweep_fast(const Cons &Cn, const double2 *hl, const double2 xr3[3],
                                           const double2 hr3[3], const double K[NCON], double L[NCON],
                                           double &v0, double &v1, double &dmax, bool &vfin) {
  ConsM Mf{Cn};
  asm volatile("" ::: "memory");  // reload the LDS slots each sweep (no hoisting)
  if (!MPCEKF_HILD_NEXTV) hild_v(hl, xr3, L, v0, v1);
  double u0 = 0.0, u1 = 0.0;
  asm volatile("" ::: "memory");
  // row i's slots are read MPCEKF_HILD_PF rows ahead: ds_read latency (~76 cycles idle,
  // more under load) stays off the chain; one row ahead left ~10 instructions between a
  // read and its use
  constexpr int PF = MPCEKF_HILD_PF;
  double2 xq[PF], hq[PF];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    xq[p] = hx_r(hl, xr3, p < NCON ? p : NCON - 1);
    hq[p] = hh_r(hl, hr3, p < NCON ? p : NCON - 1);
  }
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    const double2 xc = xq[i % PF], hc = hq[i % PF];
    if (i + PF < NCON) {
      xq[i % PF] = hx_r(hl, xr3, i + PF);
      hq[i % PF] = hh_r(hl, hr3, i + PF);
    }
    // M(i, k) entries that are structural zeros (constraintsMPC.m's Cu / I blocks and the
    // first row of each Toeplitz block) add +-0 to t: dropped here.  Exact for the fast form:
    // with v finite a +-0 term changes at most the sign of a zero t, and -t * (1/H_ii) + L_i
    // is then L_i, or +0 when L_i = +0 (round to nearest: -0 + +0 = +0), or NaN for 1/H_ii
    // infinite, either way; a non-finite v marks the sweep bad in both forms
    double t = K[i];
    if (!mzero(i, 0)) t = __builtin_fma(Mf(i, 0), v0, t);
    if (!mzero(i, 1)) t = __builtin_fma(Mf(i, 1), v1, t);
    const double m = fmin_q(t * hc.y, L[i]);   // fmin / fmax(., fabs) without the canonicalising maxes
    const double nl = L[i] - m;
    dmax = fmax_abs_q(dmax, m);
    L[i] = nl;
    v0 = __builtin_fma(-xc.x, m, v0);   // fma(x, d, v) with d = -m: the same value
    v1 = __builtin_fma(-xc.y, m, v1);
    if (MPCEKF_HILD_NEXTV) {
      u0 = __builtin_fma(xc.x, nl, u0);
      u1 = __builtin_fma(xc.y, nl, u1);
    }
  }
  vfin = isfinite(v0) && isfinite(v1);
  if (MPCEKF_HILD_NEXTV) {
    v0 = u0;
    v1 = u1;
  }
}

// The exact form for lanes the fast form flagged: plain division, v recomputed from
// lambda after a non-finite d (orc_hildreth), frozen lanes (done) keep lambda.
__device__ __forceinline__ void sweep_careful(const Cons &Cn, const double2 *hl, const double K[NCON],
                                              double L[NCON], bool done, double tol, bool &conv) {
  ConsM Mf{Cn};
  auto xv = [&](double &v0, double &v1) {
    v0 = 0.0;
    v1 = 0.0;
#pragma unroll
    for (int j = 0; j < NCON; ++j) {
      const double2 x = hx(hl, j);
      v0 = __builtin_fma(x.x, L[j], v0);
      v1 = __builtin_fma(x.y, L[j], v1);
    }
  };
  asm volatile("" ::: "memory");
  double v0, v1;
  xv(v0, v1);
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    const double2 x = hx(hl, i), hr = hh(hl, i);
    double t = __builtin_fma(Mf(i, 0), v0, K[i]);
    t = __builtin_fma(Mf(i, 1), v1, t);
    const double li = L[i];
    double nl;
    const double ds = hild_step(t, hr.x, hr.y, li, nl);
    if (!(fabs(ds) < tol)) conv = false;
    const double nli = done ? li : nl;
    const double d = done ? 0.0 : ds;
    L[i] = nli;
    if (!isfinite(d)) {
      xv(v0, v1);
    } else {
      v0 = __builtin_fma(x.x, d, v0);
      v1 = __builtin_fma(x.y, d, v1);
    }
  }
}

// The dense sweep for lanes with a non-finite X or M entry (orc_hildreth): H(i,:)*lambda
// as 4 interleaved partial sums combined as (p0 + p1) + (p2 + p3).
__device__ __forceinline__ void sweep_dense(const Cons &Cn, const XS &Xs, const double K[NCON], double L[NCON],
                                            bool done, double tol, bool &conv) {
  ConsM Mf{Cn};
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    const double m0 = Mf(i, 0), m1 = Mf(i, 1);
    double p4[4] = {0.0, 0.0, 0.0, 0.0}, hii = 0.0;
#pragma unroll
    for (int j = 0; j < NCON; ++j) {
      const double h = (0.0 + m0 * xval(Xs, j, 0)) + m1 * xval(Xs, j, 1);
      if (j == i) hii = h;
      p4[j & 3] = p4[j & 3] + h * L[j];
    }
    const double s = (p4[0] + p4[1]) + (p4[2] + p4[3]);
    const double li = L[i];
    const double w = -((K[i] + s) - hii * li) / hii;
    const double nl = w > 0 ? w : 0.0;
    if (!(fabs(nl - li) < tol)) conv = false;
    L[i] = done ? li : nl;
  }
}

// hildreth.m:32-44, lane per problem, in two launches.  Every lane of a wave stays in
// each loop until all are done: on MI355X a wave whose EXEC holds fewer than 16 lanes
// issues FP64 VALU up to 2.6x slower under full-chip load (tools/micro/exec_micro.hip).
// `done` = true makes a lane a passenger from the start (a finite dummy problem,
// nothing kept).  hl = the lane's LDS slots (HILD_LDS_PER_WAVE per wave).
//
// hild_fast (k_hild): the fast rank-2 sweep for lanes with finite X, M, every H_ii in
// hild_step's reciprocal domain and a finite warm start.  Lanes keep sweeping after they
// converge; the lambda they converged with goes to L0 (their warm start is no longer
// needed) and comes back after the loop.  A lane whose sweep ends with a non-finite v,
// and every lane outside the fast form's
// domain, returns `slow` with its warm start intact in L0: every sweep before the
// flag was bit-identical to the exact form, so restarting it with the exact rules
// gives the exact form's result.
// hild_slow (k_hild_slow, only waves holding a slow lane): sweep_careful for finite X
// and M, the dense sweep otherwise.  Kept out of k_hild so that the fast loop's
// register allocation carries none of their pressure (224 VGPRs, no AGPR traffic).
__device__ __forceinline__ bool hild_fast(const Cons &Cn, const double E[NC][NC], double L[NCON], int maxIter,
                                          double tol, const double K[NCON], bool done, double2 *hl, double *L0,
                                          int64_t l0_stride, int &nexec) {
  static_assert(NC == 2, "written for Nc = 2");
  bool fin, yok;
  {
    XS Xs;
    hild_x(Cn, E, Xs, fin);
    yok = hild_stage(Cn, Xs, hl);
  }
  double2 xr3[3], hr3[3];  // slots 0-2 (the constant rows'), the staged bits
#pragma unroll
  for (int sl = 0; sl < 3; ++sl) {
    xr3[sl] = hl[sl * 64];
    hr3[sl] = hl[(HS_X + sl) * 64];
  }
  nexec = maxIter;
  bool lok = true;
#pragma unroll
  for (int i = 0; i < NCON; ++i) lok = lok && isfinite(L[i]);
  bool slow = !done && !(fin && yok && lok);
  bool active = !done && !slow;  // still sweeping for itself
  double v0, v1;
  hild_v(hl, xr3, L, v0, v1);
#pragma unroll 1
  for (int it = 1; it <= maxIter; ++it) {
    if (__all(!active)) break;
    double dmax = 0.0;
    bool vfin;
    sweep_fast(Cn, hl, xr3, hr3, K, L, v0, v1, dmax, vfin);
    const bool bad = !vfin;
    const bool conv = dmax < tol;
    const bool newconv = active && !bad && conv;
    if (active && bad) slow = true;
    if (newconv) {
      nexec = it;
#pragma unroll
      for (int i = 0; i < NCON; ++i) L0[i * l0_stride] = L[i];
    }
    active = active && !bad && !conv;
  }
  // converged lanes take their lambda back; lanes at maxIter keep their last sweep's
  if (!active && !done && !slow) {
#pragma unroll
    for (int i = 0; i < NCON; ++i) L[i] = L0[i * l0_stride];
  }
  return slow;
}

__device__ __forceinline__ int hild_slow(const Cons &Cn, const double E[NC][NC], double L[NCON], int maxIter,
                                         double tol, const double K[NCON], bool done, double2 *hl) {
  bool fin;
  XS Xs;
  hild_x(Cn, E, Xs, fin);
  (void)hild_stage(Cn, Xs, hl);
  int nexec = maxIter;
  if (__any(fin && !done)) {
    bool cdone = done || !fin;
#pragma unroll 1
    for (int it = 1; it <= maxIter; ++it) {
      if (__all(cdone)) break;
      bool conv = true;
      sweep_careful(Cn, hl, K, L, cdone, tol, conv);
      if (!cdone && conv) {
        cdone = true;
        nexec = it;
      }
    }
  }
  if (__any(!fin && !done)) {
    bool ddone = done || fin;
#pragma unroll 1
    for (int it = 1; it <= maxIter; ++it) {
      if (__all(ddone)) break;
#pragma unroll
      for (int k = 0; k < NC; ++k) {  // opaque per sweep: no hoisting of the 529 H entries
        launder(Xs.a[k]); launder(Xs.b[k]); launder(Xs.c[k]);
#pragma unroll
        for (int i = 0; i < 3 * NP; ++i) launder(Xs.t[i][k]);
      }
      bool conv = true;
      sweep_dense(Cn, Xs, K, L, ddone, tol, conv);
      if (!ddone && conv) {
        ddone = true;
        nexec = it;
      }
    }
  }
  return nexec;
}

// M'*lambda (hildreth.m:46; the caller adds F and solves -E\(.))
__device__ __forceinline__ void hild_mtl(const Cons &Cn, const double L[NCON], double Mtl[NC]) {
  ConsM Mf{Cn};
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NCON; ++i) s = s + Mf(i, k) * L[i];
    Mtl[k] = s;
  }
}

// ---------------------------------------------------------------------------
// LDS staging
// ---------------------------------------------------------------------------
// The block's copy of a ROM blob (L2-resident, 30-130 KB) into LDS: 16 loads of 16 B per
// lane in flight before their stores.  A plain copy loop waited one L2 round trip per
// 16 B per lane (load, s_waitcnt vmcnt(0), ds_write): ~32 round trips for the cell blob.
__device__ __forceinline__ void stage_lds(double *dst, const double *src, int len) {
  constexpr int B = 16;
  const int n2 = len / 2, nt = blockDim.x;
  const double2 *s2 = reinterpret_cast<const double2 *>(src);
  double2 *d2 = reinterpret_cast<double2 *>(dst);
  int i = threadIdx.x;
  for (; i + (B - 1) * nt < n2; i += B * nt) {
    double2 v[B];
#pragma unroll
    for (int b = 0; b < B; ++b) v[b] = s2[i + b * nt];
#pragma unroll
    for (int b = 0; b < B; ++b) d2[i + b * nt] = v[b];
  }
  // The remainder: clamped loads AND clamped stores, no branch.  With guarded stores the
  // compiler sank each load into its store's branch, so the remainder (up to 15 chunks per
  // lane for the cell blob) waited one L2 round trip per chunk.  Lanes past the end store
  // the last chunk's own value to the last chunk: the same bytes, whichever lane lands.
  if (n2 > 0) {
    double2 v[B];
#pragma unroll
    for (int b = 0; b < B; ++b) v[b] = s2[min(i + b * nt, n2 - 1)];
#pragma unroll
    for (int b = 0; b < B; ++b) d2[min(i + b * nt, n2 - 1)] = v[b];
  }
  if ((len & 1) && threadIdx.x == 0) dst[len - 1] = src[len - 1];
}

// The ring inputs of a replay are loaded RCH steps at a time, all in flight together:
// a model first touched after a set-point crossing has up to LAZY_H - 1 skipped steps,
// and a load per step inside the loop waited one memory round trip each.  The FMAs then
// run in step order, so the bits are the per-step loop's.
#ifndef MPCEKF_RING_CHUNK
#define MPCEKF_RING_CHUNK 8
#endif
constexpr int RCH = MPCEKF_RING_CHUNK;
// ring[k % LAZY_H] for k = k0 .. k0 + RCH - 1 (clamped to kmax: a valid slot)
__device__ __forceinline__ void ring_chunk(const double *ring, const KState &s, int64_t c, int k0, int kmax,
                                           double v[RCH]) {
#pragma unroll
  for (int i = 0; i < RCH; ++i) v[i] = ring[(size_t)(min(k0 + i, kmax) % LAZY_H) * s.n + c];
}
// ---------------------------------------------------------------------------
// k_plant: OB_step simStep outputs for every cell (lane per cell)
// ---------------------------------------------------------------------------
template <bool GR, bool PL>
__global__ void __launch_bounds__(256) k_plant(const KRom r, const KState s, const double *iapp, double *vout,
                                               const int lazy_t, const double *tc_in) {
  extern __shared__ double lds[];
  // GR: tables only in LDS (tb + plant_tab is lds), model rows from the global blob
  const int lo = GR ? r.plant_tab : 0;
  stage_lds(lds, r.plant_blob + lo, r.plant_len - lo);
  __syncthreads();
  const double *tb = lds - lo;
  const double *L = GR ? r.plant_blob : lds;
  const double *Tp = tb + r.plant_tab + r.plant_tablen;
  const double *Zp = Tp + MAXT;
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && lazy_t) *s.hslow = 0;  // k_hild_slow of the previous step has finished
  if (c >= s.n) return;
  if (tc_in) s.Tc[c] = tc_in[c];  // this step's TC (runMPC.m:85-92), read by every later kernel
  if (lazy_t) {  // this step's inputs, for the deferred updates of every model (k_cell, k_flush)
    const size_t slot = (size_t)(lazy_t % LAZY_H) * s.n + c;
    s.hist_u[slot] = iapp[c];
    s.hist_p[slot] = s.priorI[c];
  }
  if (s.status[c] & ST_ERROR) {
    vout[c] = __builtin_nan("");
    return;
  }
  double Iapp = iapp[c];
  double T = (tc_in ? tc_in[c] : s.Tc[c]) + 273.15;  // OB_step.m:75
  const ETab et = etab<PL>(r, tb + r.plant_tab, T);
  double SOCnAvg = s.SOCn[c], SOCpAvg = s.SOCp[c];
  const double negSOC = SOCnAvg, posSOC = SOCpAvg;  // obs.negSOC / posSOC: pre-update (OB_step.m:226-227)
  double cellSOC = (SOCnAvg - r.th0n) / (r.th100n - r.th0n);
  const double Cdleffn = et.f(0, EF_CDL, s.SOC0n[c]), Cdleffp = et.f(1, EF_CDL, s.SOC0p[c]);  // OB_step.m:212-219
  double dUn = et.f(0, EF_DU, SOCnAvg), dUp = et.f(1, EF_DU, SOCpAvg);
  double dQn = fabs(r.th100n - r.th0n), dQp = fabs(r.th100p - r.th0p);
  double res0n = -dQn / (3600 * r.Q - Cdleffn * dQn * dUn);
  double res0p = dQp / (3600 * r.Q - Cdleffp * dQp * dUp);
  SOCnAvg = SOCnAvg + res0n * Iapp * r.Ts;
  SOCpAvg = SOCpAvg + res0p * Iapp * r.Ts;
  if (SOCnAvg < 0) SOCnAvg = 0;
  if (SOCnAvg > 1) SOCnAvg = 1;
  if (SOCpAvg < 0) SOCpAvg = 0;
  if (SOCpAvg > 1) SOCpAvg = 1;
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (r.nZ > 1) {
    int a, b;
    two_nearest(Zp, r.nZ, cellSOC, a, b);
    iZu = a > b ? a : b; iZl = a < b ? a : b;
  }
  if (r.nT > 1) {
    int a, b;
    two_nearest(Tp, r.nT, T, a, b);
    iTu = a > b ? a : b; iTl = a < b ? a : b;
  }
  double Zu = Zp[iZu], Zl = Zp[iZl], Tu = Tp[iTu], Tl = Tp[iTl];
  int mm[4] = {iTl * r.nZ + iZl, iTl * r.nZ + iZu, iTu * r.nZ + iZl, iTu * r.nZ + iZu};
  double y[4][NPLANT];
  double *bx = s.bigx + (size_t)c * r.NM * 6;
  // the 4 corner states as of step t-1: all loads before any store (duplicate corners)
  double xs[4][6];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double2 *p = reinterpret_cast<const double2 *>(bx + (size_t)mm[j] * 6);
    double2 q0 = p[0], q1 = p[1], q2 = p[2];
    xs[j][0] = q0.x; xs[j][1] = q0.y; xs[j][2] = q1.x; xs[j][3] = q1.y; xs[j][4] = q2.x; xs[j][5] = q2.y;
  }
  int tsj[4] = {0, 0, 0, 0};
  if (lazy_t) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tsj[j] = s.ts_plant[c * r.NM + mm[j]];
      const double *a = L + mm[j] * PREC + NPLANT * NX + 2 * NPLANT;
      for (int k = tsj[j] + 1; k < lazy_t; ++k) {  // OB_step.m:198-200 for the skipped steps
        const double u = s.hist_u[(size_t)(k % LAZY_H) * s.n + c];
#pragma unroll
        for (int e = 0; e < 6; ++e) xs[j][e] = __builtin_fma(a[e], xs[j][e], u);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double x[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) x[e] = xs[j][e];
    const double *B = L + mm[j] * PREC;
#pragma unroll
    for (int q = 0; q < NPLANT; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < NX; ++k) acc = acc + B[q * NX + k] * x[k];
      acc = acc + B[NPLANT * NX + q] * x[5];
      y[j][q] = acc + B[NPLANT * NX + NPLANT + q] * Iapp;
      launder(y[j][q]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  double aZ = 0.0, aT = 0.0;
  if (Zu != Zl) aZ = (cellSOC - Zl) / (Zu - Zl);
  if (Tu != Tl) aT = (T - Tl) / (Tu - Tl);
  double yk[NPLANT];
#pragma unroll
  for (int q = 0; q < NPLANT; ++q)
    yk[q] = (1 - aT) * ((1 - aZ) * y[0][q] + aZ * y[1][q]) + aT * ((1 - aZ) * y[2][q] + aZ * y[3][q]);
  double th0 = fmin(fmax(yk[R_TH0] + s.SOC0n[c], 1e-6), 1 - 1e-6);
  double th3 = fmin(fmax(yk[R_TH3] + s.SOC0p[c], 1e-6), 1 - 1e-6);
  double te1 = fmax(yk[R_TE1] + 1, 1e-6);
  double teE = fmax(yk[R_TEE] + 1, 1e-6);
  double i0n = et.f(0, EF_K0, negSOC) * sqrt(te1 * (1 - th0) * th0);  // OB_step.m:329-332
  double i0p = et.f(1, EF_K0, posSOC) * sqrt(teE * (1 - th3) * th3);
  double negEta0 = 2 * r.R * T / r.F * dasinh(yk[R_IF0] / (2 * i0n));
  double posEta3 = 2 * r.R * T / r.F * dasinh(yk[R_IF3] / (2 * i0p));
  double Uocpn0 = et.f(0, EF_U, th0), Uocpp3 = et.f(1, EF_U, th3);
  const double Rfn = et.f(0, EF_RF, negSOC), Rfp = et.f(1, EF_RF, posSOC);  // OB_step.m:339-340
  double V = posEta3 - negEta0 + yk[R_PHIE] + Uocpp3 - Uocpn0 + (Rfp * yk[R_IFDL3] - Rfn * yk[R_IFDL0]);
  V = V - r.Rc * Iapp;
  s.SOCn[c] = SOCnAvg;
  s.SOCp[c] = SOCpAvg;
  vout[c] = V;
  if (lazy_t) {  // advance the corners through step t in place (eager mode: k_bulk does all models)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (tsj[j] >= lazy_t) continue;
      const double *a = L + mm[j] * PREC + NPLANT * NX + 2 * NPLANT;
      double2 *p = reinterpret_cast<double2 *>(bx + (size_t)mm[j] * 6);
      double x[6];
#pragma unroll
      for (int e = 0; e < 6; ++e) x[e] = __builtin_fma(a[e], xs[j][e], Iapp);
      p[0] = make_double2(x[0], x[1]);
      p[1] = make_double2(x[2], x[3]);
      p[2] = make_double2(x[4], x[5]);
      s.ts_plant[c * r.NM + mm[j]] = lazy_t;
    }
  }
}

// ---------------------------------------------------------------------------
// k_plant4: k_plant with a lane quad per cell, lane j = corner j of OB_step.m:251-275.
// Lane-per-cell k_plant runs 65,536 cells as one wave per SIMD, so every round trip
// (the per-cell scalars, then the corner gathers they select) and every dependent FP64
// chain is exposed (60 % of its cycles in s_waitcnt, VALU 15 %).  Here lane j gathers and
// replays only its corner's 48-B state and forms its 9 output rows; the blend of
// OB_step.m:281-285 takes the four corners' rows by DPP quad broadcasts in the one-lane
// expression order, and the per-cell scalar chain (bracket, clamps, asinh, Vcell) is the
// same instruction stream for the whole quad.  1024-thread blocks: 256 cells share one
// staged plant blob per CU at 4 waves per SIMD.  Results: k_plant's bits.
// ---------------------------------------------------------------------------
#ifndef MPCEKF_PLANT_QUAD
#define MPCEKF_PLANT_QUAD 1
#endif
constexpr int PLANT4_BLOCK = 1024;
template <bool GR, bool PL>
__global__ void __launch_bounds__(PLANT4_BLOCK) k_plant4(const KRom r, const KState s, const double *iapp,
                                                         double *vout, const int lazy_t, const double *tc_in) {
  extern __shared__ double lds[];
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = (int)(gt & 3);
  const int64_t c = gt >> 2;  // a quad is one cell: every exit below is quad-uniform
#ifdef MPCEKF_STAMPS
  if (c < s.n && j == 0 && s.stamps) s.stamps[(size_t)19 * s.n + c] = (long long)__builtin_amdgcn_s_memtime();
#endif
  const int lo = GR ? r.plant_tab : 0;
  stage_lds(lds, r.plant_blob + lo, r.plant_len - lo);
  __syncthreads();
  const double *tb = lds - lo;
  const double *L = GR ? r.plant_blob : lds;
  const double *Tp = tb + r.plant_tab + r.plant_tablen;
  const double *Zp = Tp + MAXT;
  if (gt == 0 && lazy_t) *s.hslow = 0;  // k_hild_slow of the previous step has finished
  if (c >= s.n) return;
  STAMPP(0);
  const double Iapp = iapp[c];
  const double tcs = tc_in ? tc_in[c] : s.Tc[c];
  const double priorI = s.priorI[c];
  const int status = s.status[c];
  double SOCnAvg = s.SOCn[c], SOCpAvg = s.SOCp[c];
  const double SOC0n = s.SOC0n[c], SOC0p = s.SOC0p[c];
  if (j == 0) {
    if (tc_in) s.Tc[c] = tcs;  // this step's TC (runMPC.m:85-92), read by every later kernel
    if (lazy_t) {  // this step's inputs, for the deferred updates of every model (k_cell, k_flush)
      const size_t slot = (size_t)(lazy_t % LAZY_H) * s.n + c;
      s.hist_u[slot] = Iapp;
      s.hist_p[slot] = priorI;
    }
  }
  if (status & ST_ERROR) {
    if (j == 0) vout[c] = __builtin_nan("");
    return;
  }
  const double T = tcs + 273.15;  // OB_step.m:75
  const ETab et = etab<PL>(r, tb + r.plant_tab, T);
  const double negSOC = SOCnAvg, posSOC = SOCpAvg;  // obs.negSOC / posSOC: pre-update (OB_step.m:226-227)
  double cellSOC = (SOCnAvg - r.th0n) / (r.th100n - r.th0n);
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (r.nZ > 1) {
    int a, b;
    two_nearest(Zp, r.nZ, cellSOC, a, b);
    iZu = a > b ? a : b; iZl = a < b ? a : b;
  }
  if (r.nT > 1) {
    int a, b;
    two_nearest(Tp, r.nT, T, a, b);
    iTu = a > b ? a : b; iTl = a < b ? a : b;
  }
  STAMPP(1);
  // this lane's corner: mm = {Tl Zl, Tl Zu, Tu Zl, Tu Zu}[j]
  const int mj = ((j & 2) ? iTu : iTl) * r.nZ + ((j & 1) ? iZu : iZl);
  double *bx = s.bigx + ((size_t)c * r.NM + mj) * 6;
  double xs[6];
  {
    const double2 *p = reinterpret_cast<const double2 *>(bx);
    const double2 q0 = p[0], q1 = p[1], q2 = p[2];
    xs[0] = q0.x; xs[1] = q0.y; xs[2] = q1.x; xs[3] = q1.y; xs[4] = q2.x; xs[5] = q2.y;
  }
  const int tsj = lazy_t ? s.ts_plant[c * r.NM + mj] : 0;
  // the per-cell scalar chain runs while the corner gathers are in flight
  const double Cdleffn = et.f(0, EF_CDL, SOC0n), Cdleffp = et.f(1, EF_CDL, SOC0p);  // OB_step.m:212-219
  double dUn = et.f(0, EF_DU, SOCnAvg), dUp = et.f(1, EF_DU, SOCpAvg);
  double dQn = fabs(r.th100n - r.th0n), dQp = fabs(r.th100p - r.th0p);
  double res0n = -dQn / (3600 * r.Q - Cdleffn * dQn * dUn);
  double res0p = dQp / (3600 * r.Q - Cdleffp * dQp * dUp);
  SOCnAvg = SOCnAvg + res0n * Iapp * r.Ts;
  SOCpAvg = SOCpAvg + res0p * Iapp * r.Ts;
  if (SOCnAvg < 0) SOCnAvg = 0;
  if (SOCnAvg > 1) SOCnAvg = 1;
  if (SOCpAvg < 0) SOCpAvg = 0;
  if (SOCpAvg > 1) SOCpAvg = 1;
  const double Zu = Zp[iZu], Zl = Zp[iZl], Tu = Tp[iTu], Tl = Tp[iTl];
  double aZ = 0.0, aT = 0.0;
  if (Zu != Zl) aZ = (cellSOC - Zl) / (Zu - Zl);
  if (Tu != Tl) aT = (T - Tl) / (Tu - Tl);
  STAMPP(2);
  const double *a = L + mj * PREC + NPLANT * NX + 2 * NPLANT;
  if (lazy_t)  // OB_step.m:198-200 for the skipped steps, RCH ring inputs per round trip
    for (int k0 = tsj + 1; k0 < lazy_t; k0 += RCH) {
      double u[RCH];
      ring_chunk(s.hist_u, s, c, k0, lazy_t - 1, u);
#pragma unroll
      for (int i = 0; i < RCH; ++i)
        if (k0 + i < lazy_t)
#pragma unroll
          for (int e = 0; e < 6; ++e) xs[e] = __builtin_fma(a[e], xs[e], u[i]);
    }
  STAMPP(3);
  const double *B = L + mj * PREC;
  double yk[NPLANT];
#pragma unroll
  for (int q = 0; q < NPLANT; ++q) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k) acc = acc + B[q * NX + k] * xs[k];
    acc = acc + B[NPLANT * NX + q] * xs[5];
    const double y = acc + B[NPLANT * NX + NPLANT + q] * Iapp;
    const double y0 = qbc<0>(y), y1 = qbc<1>(y), y2 = qbc<2>(y), y3 = qbc<3>(y);
    yk[q] = (1 - aT) * ((1 - aZ) * y0 + aZ * y1) + aT * ((1 - aZ) * y2 + aZ * y3);
    __builtin_amdgcn_sched_barrier(0);  // one row's LDS operands at a time: 128 VGPRs at 4 waves/SIMD
  }
  STAMPP(4);
  double th0 = fmin(fmax(yk[R_TH0] + SOC0n, 1e-6), 1 - 1e-6);
  double th3 = fmin(fmax(yk[R_TH3] + SOC0p, 1e-6), 1 - 1e-6);
  double te1 = fmax(yk[R_TE1] + 1, 1e-6);
  double teE = fmax(yk[R_TEE] + 1, 1e-6);
  double i0n = et.f(0, EF_K0, negSOC) * sqrt(te1 * (1 - th0) * th0);  // OB_step.m:329-332
  double i0p = et.f(1, EF_K0, posSOC) * sqrt(teE * (1 - th3) * th3);
  double negEta0 = 2 * r.R * T / r.F * dasinh(yk[R_IF0] / (2 * i0n));
  double posEta3 = 2 * r.R * T / r.F * dasinh(yk[R_IF3] / (2 * i0p));
  double Uocpn0 = et.f(0, EF_U, th0), Uocpp3 = et.f(1, EF_U, th3);
  const double Rfn = et.f(0, EF_RF, negSOC), Rfp = et.f(1, EF_RF, posSOC);  // OB_step.m:339-340
  double V = posEta3 - negEta0 + yk[R_PHIE] + Uocpp3 - Uocpn0 + (Rfp * yk[R_IFDL3] - Rfn * yk[R_IFDL0]);
  V = V - r.Rc * Iapp;
  STAMPP(5);
  if (j == 0) {
    s.SOCn[c] = SOCnAvg;
    s.SOCp[c] = SOCpAvg;
    vout[c] = V;
  }
  // advance this corner through step t in place (eager mode: k_bulk does all models); a
  // duplicate corner (single-set-point grids) is written by two lanes with the same bits
  if (lazy_t && tsj < lazy_t) {
    double2 *p = reinterpret_cast<double2 *>(bx);
    double x[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) x[e] = __builtin_fma(a[e], xs[e], Iapp);
    p[0] = make_double2(x[0], x[1]);
    p[1] = make_double2(x[2], x[3]);
    p[2] = make_double2(x[4], x[5]);
    s.ts_plant[c * r.NM + mj] = lazy_t;
  }
  STAMPP(6);
}

// ---------------------------------------------------------------------------
// k_bulk: all-model plant advance and EKF time update (HBM streaming)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_bulk(const KRom r, const KCfg cf, const KState s, const double *iapp,
                                              int do_plant, int do_ekf) {
  extern __shared__ double lds[];
  const int NM = r.NM;
  const int ne = NM * REC, np = NM * 6;
  stage_lds(lds, r.bulk_tab, ne + np);
  __syncthreads();
  const double *cC = lds, *cP = lds + ne;
  const double W = cf.SigmaW;
  for (int64_t c = blockIdx.x; c < s.n; c += gridDim.x) {
    if (do_ekf) {
      double pri = s.priorI[c];
      double2 *base = reinterpret_cast<double2 *>(s.ekf + (size_t)c * ne);
      for (int j = threadIdx.x; j < ne / 2; j += blockDim.x) {
        int e0 = (2 * j) % REC;
        double2 v = base[j];
        double add0 = e0 < NX ? pri : W;
        double add1 = e0 + 1 < NX ? pri : W;
        v.x = __builtin_fma(cC[2 * j], v.x, add0);
        v.y = __builtin_fma(cC[2 * j + 1], v.y, add1);
        base[j] = v;
      }
    }
    if (do_plant) {
      double u = iapp[c];
      double2 *base = reinterpret_cast<double2 *>(s.bigx + (size_t)c * np);
      for (int j = threadIdx.x; j < np / 2; j += blockDim.x) {
        double2 v = base[j];
        v.x = __builtin_fma(cP[2 * j], v.x, u);
        v.y = __builtin_fma(cP[2 * j + 1], v.y, u);
        base[j] = v;
      }
    }
  }
}

// k_flush: brings every local model (EKF record and plant state) of every cell
// from its timestamp to step t with the logged inputs, then stamps it new_ts.
// Block per cell, the cell's input rings and timestamps staged in LDS.
// Lane per model: a wave takes one cell at a time (grid-stride) with its lanes on
// models m0 + lane; the model's coefficients (diag(A) for xhat, a_p a_q for Sigma, bigA
// for the plant) stay in registers across cells, the record (26 doubles) is loaded once,
// replayed step by step and stored once.  The step inputs come from the lane holding
// that ring slot (readlane; k is wave-uniform), so a step is 26 FMAs and no memory.
__device__ __forceinline__ double rl64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__global__ void __launch_bounds__(256) k_flush(const KRom r, const KCfg cf, const KState s, const int t,
                                               const int new_ts, const int64_t c_lo, const int64_t c_hi) {
  const int NM = r.NM;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const double W = cf.SigmaW;
  const double *cC = r.bulk_tab, *cP = r.bulk_tab + (size_t)NM * REC;
  for (int m0 = 0; m0 < NM; m0 += 64) {
    const int m = m0 + lane;
    const bool act = m < NM;
    const int mm = act ? m : NM - 1;
    double ce[REC], cp[6];
#pragma unroll
    for (int e = 0; e < REC; ++e) ce[e] = cC[(size_t)mm * REC + e];
#pragma unroll
    for (int e = 0; e < 6; ++e) cp[e] = cP[(size_t)mm * 6 + e];
    // software pipelined over the wave's cells: the next cell's rings, timestamps and
    // records are loaded while this cell replays, so every wave keeps a cell's 13.6 KB
    // in flight (MPCEKF_FLUSH_PF = 0: load, replay, store in turn)
    struct FCell {
      double hpl, hul, xe[REC], xp[6];
      int tse, tsp;
    };
    auto fload = [&](int64_t c, FCell &F) {
      F.hpl = s.hist_p[(size_t)(lane & (LAZY_H - 1)) * s.n + c];
      F.hul = s.hist_u[(size_t)(lane & (LAZY_H - 1)) * s.n + c];
      // MB never time-updates the per-model EKF records (iterEKF.m:90-102)
      F.tse = (act && !(cf.flags & KF_MB)) ? s.ts_ekf[c * NM + m] : t;
      F.tsp = act ? s.ts_plant[c * NM + m] : t;
      const double2 *re = reinterpret_cast<const double2 *>(s.ekf + ((size_t)c * NM + mm) * REC);
      const double2 *rp = reinterpret_cast<const double2 *>(s.bigx + ((size_t)c * NM + mm) * 6);
#pragma unroll
      for (int e = 0; e < REC / 2; ++e) {
        const double2 v = re[e];
        F.xe[2 * e] = v.x;
        F.xe[2 * e + 1] = v.y;
      }
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const double2 v = rp[e];
        F.xp[2 * e] = v.x;
        F.xp[2 * e + 1] = v.y;
      }
    };
    FCell cur;
    if (MPCEKF_FLUSH_PF && c_lo + w0 < c_hi) fload(c_lo + w0, cur);
    for (int64_t c = c_lo + w0; c < c_hi; c += nw) {
      FCell nx;
      if (MPCEKF_FLUSH_PF) {
        if (c + nw < c_hi) fload(c + nw, nx);
      } else {
        fload(c, cur);
      }
      const double hpl = cur.hpl, hul = cur.hul;
      const int tse = cur.tse, tsp = cur.tsp;
      double2 *re = reinterpret_cast<double2 *>(s.ekf + ((size_t)c * NM + mm) * REC);
      double2 *rp = reinterpret_cast<double2 *>(s.bigx + ((size_t)c * NM + mm) * 6);
      double *xe = cur.xe, *xp = cur.xp;
      int kmin = min(tse, tsp);
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) kmin = min(kmin, __shfl_xor(kmin, o));
      for (int k = kmin + 1; k <= t; ++k) {  // k is wave-uniform
        const int sl = k & (LAZY_H - 1);
        const double p = rl64(hpl, sl), u = rl64(hul, sl);
        if (k > tse) {
#pragma unroll
          for (int e = 0; e < NX; ++e) xe[e] = __builtin_fma(ce[e], xe[e], p);
#pragma unroll
          for (int e = NX; e < REC; ++e) xe[e] = __builtin_fma(ce[e], xe[e], W);
        }
        if (k > tsp) {
#pragma unroll
          for (int e = 0; e < 6; ++e) xp[e] = __builtin_fma(cp[e], xp[e], u);
        }
      }
      if (tse < t) {
#pragma unroll
        for (int e = 0; e < REC / 2; ++e) re[e] = make_double2(xe[2 * e], xe[2 * e + 1]);
      }
      if (tsp < t) {
#pragma unroll
        for (int e = 0; e < 3; ++e) rp[e] = make_double2(xp[2 * e], xp[2 * e + 1]);
      }
      if (act) {
        s.ts_ekf[c * NM + m] = new_ts;
        s.ts_plant[c * NM + m] = new_ts;
      }
      if (MPCEKF_FLUSH_PF) cur = nx;
    }
  }
}

// k_flush_coal: k_flush with coalesced record traffic (NM <= 64).  A cell's EKF records
// ([NM][20] doubles) and plant states ([NM][6]) are contiguous, and every element's update
// is its own recurrence x <- fma(coef, x, input) over the steps its model skipped, so a wave
// takes the cell's regions as consecutive 16-byte chunks, lane l chunk l + 64 q: each load
// and store instruction moves one contiguous KB instead of 16 B at a 160-B stride per lane.
// A chunk is two elements of one model (REC and 6 are even); its coefficients are at the
// same offset of bulk_tab, its timestamp is the model's.  Same fmas, same order per element.
// Bitwise-green but slower (645 vs 455 us per flush at configs[2], profiles/r03n_ab_flush_coal.txt):
// 13 per-chunk timestamp gathers and a compare per chunk and step replace k_flush's two per
// lane, and the per-lane 16-B stride was not what held k_flush back.  Off by default.
constexpr int FC_QE = 10, FC_QP = 3;  // chunks per lane: 64 * 10 >= 64 * 20 / 2, 64 * 3 >= 64 * 6 / 2
__global__ void __launch_bounds__(256) k_flush_coal(const KRom r, const KCfg cf, const KState s, const int t,
                                                    const int new_ts, const int64_t c_lo, const int64_t c_hi) {
  const int NM = r.NM;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const double W = cf.SigmaW;
  const bool mb = cf.flags & KF_MB;  // MB never time-updates the per-model EKF records
  const int ne2 = NM * REC / 2, np2 = NM * 3;
  const double *cC = r.bulk_tab, *cP = r.bulk_tab + (size_t)NM * REC;
  // per-lane constants: the chunks' coefficients, models and element kinds
  double2 ke[FC_QE], kp[FC_QP];
  int me[FC_QE], mp[FC_QP];
  bool xe0[FC_QE], xe1[FC_QE];  // element is an xhat entry (input priorI) or Sigma (input SigmaW)
#pragma unroll
  for (int q = 0; q < FC_QE; ++q) {
    const int j = lane + 64 * q, jj = j < ne2 ? j : ne2 - 1;
    ke[q] = reinterpret_cast<const double2 *>(cC)[jj];
    me[q] = j < ne2 ? (2 * j) / REC : -1;
    xe0[q] = (2 * jj) % REC < NX;
    xe1[q] = (2 * jj + 1) % REC < NX;
  }
#pragma unroll
  for (int q = 0; q < FC_QP; ++q) {
    const int j = lane + 64 * q, jj = j < np2 ? j : np2 - 1;
    kp[q] = reinterpret_cast<const double2 *>(cP)[jj];
    mp[q] = j < np2 ? (2 * j) / 6 : -1;
  }
  struct FCell {
    double hpl, hul;
    double2 xe[FC_QE], xp[FC_QP];
    int tse[FC_QE], tsp[FC_QP];
  };
  auto fload = [&](int64_t c, FCell &F) {
    F.hpl = s.hist_p[(size_t)(lane & (LAZY_H - 1)) * s.n + c];
    F.hul = s.hist_u[(size_t)(lane & (LAZY_H - 1)) * s.n + c];
    const double2 *re = reinterpret_cast<const double2 *>(s.ekf + (size_t)c * NM * REC);
    const double2 *rp = reinterpret_cast<const double2 *>(s.bigx + (size_t)c * NM * 6);
#pragma unroll
    for (int q = 0; q < FC_QE; ++q) {
      const bool a = me[q] >= 0;
      F.xe[q] = re[a ? lane + 64 * q : 0];
      F.tse[q] = (a && !mb) ? s.ts_ekf[c * NM + me[q]] : t;
    }
#pragma unroll
    for (int q = 0; q < FC_QP; ++q) {
      const bool a = mp[q] >= 0;
      F.xp[q] = rp[a ? lane + 64 * q : 0];
      F.tsp[q] = a ? s.ts_plant[c * NM + mp[q]] : t;
    }
  };
  FCell cur;
  if (c_lo + w0 < c_hi) fload(c_lo + w0, cur);
  for (int64_t c = c_lo + w0; c < c_hi; c += nw) {
    FCell nx;
    if (c + nw < c_hi) fload(c + nw, nx);
    int kmin = t;
#pragma unroll
    for (int q = 0; q < FC_QE; ++q) kmin = min(kmin, cur.tse[q]);
#pragma unroll
    for (int q = 0; q < FC_QP; ++q) kmin = min(kmin, cur.tsp[q]);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) kmin = min(kmin, __shfl_xor(kmin, o));
    for (int k = kmin + 1; k <= t; ++k) {  // k is wave-uniform
      const int sl = k & (LAZY_H - 1);
      const double p = rl64(cur.hpl, sl), u = rl64(cur.hul, sl);
#pragma unroll
      for (int q = 0; q < FC_QE; ++q)
        if (k > cur.tse[q]) {
          cur.xe[q].x = __builtin_fma(ke[q].x, cur.xe[q].x, xe0[q] ? p : W);
          cur.xe[q].y = __builtin_fma(ke[q].y, cur.xe[q].y, xe1[q] ? p : W);
        }
#pragma unroll
      for (int q = 0; q < FC_QP; ++q)
        if (k > cur.tsp[q]) {
          cur.xp[q].x = __builtin_fma(kp[q].x, cur.xp[q].x, u);
          cur.xp[q].y = __builtin_fma(kp[q].y, cur.xp[q].y, u);
        }
    }
    double2 *re = reinterpret_cast<double2 *>(s.ekf + (size_t)c * NM * REC);
    double2 *rp = reinterpret_cast<double2 *>(s.bigx + (size_t)c * NM * 6);
#pragma unroll
    for (int q = 0; q < FC_QE; ++q)
      if (me[q] >= 0 && cur.tse[q] < t) re[lane + 64 * q] = cur.xe[q];
#pragma unroll
    for (int q = 0; q < FC_QP; ++q)
      if (mp[q] >= 0 && cur.tsp[q] < t) rp[lane + 64 * q] = cur.xp[q];
    if (lane < NM) {
      s.ts_ekf[c * NM + lane] = new_ts;
      s.ts_plant[c * NM + lane] = new_ts;
    }
    cur = nx;
  }
}

// ---------------------------------------------------------------------------
// Deferred time update (fused mpcekf_step): iterEKF.m:73-84 for the steps model m
// skipped, replayed in the per-step order of the eager update (k_bulk / the oracle),
// so the record is bit-identical to one advanced every step.
// ---------------------------------------------------------------------------
// The skipped time updates of one model, steps ts+1..t (pt = the step-t input).
__device__ __forceinline__ void replay_x(double x[NX], const double *a, int ts, int t, double pt, const KState &s,
                                        int64_t c) {
  if (ts + 1 < t) {  // steps before t: their inputs from the ring
    for (int k0 = ts + 1; k0 < t; k0 += RCH) {
      double p[RCH];
      ring_chunk(s.hist_p, s, c, k0, t - 1, p);
#pragma unroll
      for (int i = 0; i < RCH; ++i)
        if (k0 + i < t)
#pragma unroll
          for (int e = 0; e < NX; ++e) x[e] = __builtin_fma(a[e], x[e], p[i]);
    }
  }
  if (ts < t)
#pragma unroll
    for (int e = 0; e < NX; ++e) x[e] = __builtin_fma(a[e], x[e], pt);
}
// a: the model's diag(A) [NX] followed by its a_p a_q coefficients [NPK] (cell blob)
__device__ __forceinline__ void replay_S(double S[NPK], const double *a, int ts, int t, double W) {
  for (int k = ts + 1; k <= t; ++k) {
#pragma unroll
    for (int i = 0, pp = 0; pp < NX; ++pp)
#pragma unroll
      for (int q = pp; q < NX; ++q, ++i) S[i] = __builtin_fma(a[NX + i], S[i], W);
  }
}

template <int NZ>
__device__ __forceinline__ void ekf_catch_up4(const KState &s, const CellCtx &cc, int NM, const int m[4], int64_t c,
                                              int t, double W, double pt) {
  // all timestamps, then all lagging records, in flight together (latency, not bytes,
  // is the cost here); a model named by several corners is advanced once
  int ts[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ts[j] = s.ts_ekf[c * NM + m[j]];
  bool need[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    need[j] = ts[j] < t;
#pragma unroll
    for (int i = 0; i < j; ++i) need[j] = need[j] && m[i] != m[j];
  }
  if (!(need[0] || need[1] || need[2] || need[3])) return;
  // pt: step t's input (the ring's slot t, which k_cell may not have stored yet: MPCEKF_RING_LATE)
  double x[4][NX], S[4][NPK];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (need[j]) load_rec(cc.erec + (size_t)m[j] * REC, x[j], S[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!need[j]) continue;
    const double *a = cc.L + m[j] * cc.stride + NZ * NX + NZ;  // diag(A) of the model (cell blob)
    for (int k0 = ts[j] + 1; k0 <= t; k0 += RCH) {
      double p[RCH];
      if (k0 < t) ring_chunk(s.hist_p, s, c, k0, t - 1, p);
#pragma unroll
      for (int i = 0; i < RCH; ++i) {
        const int k = k0 + i;
        if (k > t) break;
        const double pk_ = k == t ? pt : p[i];
#pragma unroll
        for (int e = 0; e < NX; ++e) x[j][e] = __builtin_fma(a[e], x[j][e], pk_);
#pragma unroll
        for (int q = 0; q < NPK; ++q) S[j][q] = __builtin_fma(a[NX + q], S[j][q], W);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (need[j]) {
      store_rec(cc.erec + (size_t)m[j] * REC, x[j], S[j]);
      s.ts_ekf[c * NM + m[j]] = t;
    }
}

// ---------------------------------------------------------------------------
// Model blend ('MB', initKF.m:44-49): one blended model per cell, its (n+1) state and
// full 6x6 covariance in s.mb [n][MBREC] = xhat[0..4], -, Sigma 6x6 row-major; the
// integrator xhat(end) lives in s.x0.  The sequence is oracle/mpcekf_oracle.c
// ekf_step_mb / meas_cov_mb / get_chat_v_mb, operation for operation.
// ---------------------------------------------------------------------------
constexpr int NA6 = NX + 1;
constexpr int NPK6 = NA6 * (NA6 + 1) / 2;
__device__ __forceinline__ int pk6(int r, int c) {
  return r <= c ? r * NA6 - (r * (r - 1)) / 2 + (c - r) : c * NA6 - (c * (c - 1)) / 2 + (r - c);
}

// getChatV 'MB' (iterEKF.m:448-459, 475-479, 489-491, 512-517): the gamma-weighted sums
// of the four corners' rows, then the terms; the integrator entry last.
template <int NZ>
__device__ __forceinline__ void chat_mb(const KRom &r, const CellCtx &cc, const XI &xi, double xSOC, double zTE1,
                                        double zTH0, double zTEE, double zTH3, double ChV[NA6]) {
  const ChatK K = chat_k(r, cc, xSOC, zTE1, zTH0, zTEE, zTH3);
  constexpr int rows[7] = {R_IFDL3, R_IFDL0, R_IF3, R_IF0, R_PHIE, R_TH3, R_TH0};
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    double sum[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) a = a + xi.g[j] * cc.L[xi.m[j] * cc.stride + rows[t] * NX + k];
      sum[t] = a;
    }
    double v = K.Rfp * sum[0] - K.Rfn * sum[1];
    v = v + K.Rctp * sum[2] - K.Rctn * sum[3];
    v = v + sum[4];
    v = v + K.dUp3 * sum[5] - K.dUn0 * sum[6];
    ChV[k] = v;
  }
  ChV[NX] = chat0(r, K);
}

// row' * Sigma * row on the full 6x6 (orc qform_full): t_c = sum_k fma(S_kc, row_k),
// acc = sum_c fma(t_c, row_c)
__device__ __forceinline__ double qform6(const double S[NA6 * NA6], const double row[NA6]) {
  double acc = 0.0;
#pragma unroll
  for (int cI = 0; cI < NA6; ++cI) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < NA6; ++k) t = __builtin_fma(S[k * NA6 + cI], row[k], t);
    acc = __builtin_fma(t, row[cI], acc);
  }
  return acc;
}

__device__ __forceinline__ bool is_pd6(const double a[NPK6]) {  // orc is_pd_n(6)
  double l[NA6][NA6], d[NA6];
  bool pd = true;
#pragma unroll
  for (int j = 0; j < NA6; ++j) {
    double sj = a[pk6(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) sj = __builtin_fma(-(l[j][k] * l[j][k]), d[k], sj);
    pd = pd && (sj > 0);
    d[j] = sj;
    const double inv = 1.0 / sj;
#pragma unroll
    for (int i = j + 1; i < NA6; ++i) {
      double t = a[pk6(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) t = __builtin_fma(-(l[i][k] * l[j][k]), d[k], t);
      l[i][j] = t * inv;
    }
  }
  return pd;
}

__device__ __noinline__ void jacobi6(double a[NPK6], double V[NA6 * NA6]) {  // orc_jacobi(6), packed
#pragma unroll
  for (int i = 0; i < NA6 * NA6; ++i) V[i] = (i % (NA6 + 1)) == 0 ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0, dg = 0.0;
#pragma unroll
    for (int p = 0; p < NA6; ++p) {
      dg = dg + a[pk6(p, p)] * a[pk6(p, p)];
#pragma unroll
      for (int q = p + 1; q < NA6; ++q) off = off + a[pk6(p, q)] * a[pk6(p, q)];
    }
    if (!(off > 1e-36 * dg)) break;
#pragma unroll
    for (int p = 0; p < NA6 - 1; ++p) {
#pragma unroll
      for (int q = p + 1; q < NA6; ++q) {
        double apq = a[pk6(p, q)];
        if (apq != 0.0) {
          double theta = (a[pk6(q, q)] - a[pk6(p, p)]) / (2.0 * apq);
          double t;
          if (fabs(theta) > 1e150) {
            t = 0.5 / theta;
          } else {
            t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
            if (theta < 0) t = -t;
          }
          double c = 1.0 / sqrt(t * t + 1.0), sn = t * c, tau = sn / (1.0 + c);
          a[pk6(p, p)] = a[pk6(p, p)] - t * apq;
          a[pk6(q, q)] = a[pk6(q, q)] + t * apq;
          a[pk6(p, q)] = 0.0;
#pragma unroll
          for (int rr = 0; rr < NA6; ++rr) {
            if (rr == p || rr == q) continue;
            double g = a[pk6(rr, p)], h = a[pk6(rr, q)];
            a[pk6(rr, p)] = g - sn * (h + g * tau);
            a[pk6(rr, q)] = h + sn * (g - h * tau);
          }
#pragma unroll
          for (int rr = 0; rr < NA6; ++rr) {
            double g = V[rr * NA6 + p], h = V[rr * NA6 + q];
            V[rr * NA6 + p] = g - sn * (h + g * tau);
            V[rr * NA6 + q] = h + sn * (g - h * tau);
          }
        }
      }
    }
  }
}

// iterEKF.m:164-173 on the full MB covariance (orc meas_cov_mb)
__device__ __forceinline__ void meas_cov_mb(double S[NA6 * NA6], const double L[NA6], double St, bool bump) {
  double P[NA6 * NA6], a[NPK6];
#pragma unroll
  for (int rr = 0; rr < NA6; ++rr)
#pragma unroll
    for (int cI = 0; cI < NA6; ++cI) P[rr * NA6 + cI] = __builtin_fma(-(L[rr] * St), L[cI], S[rr * NA6 + cI]);
#pragma unroll
  for (int rr = 0; rr < NA6; ++rr)
#pragma unroll
    for (int cI = rr; cI < NA6; ++cI) a[pk6(rr, cI)] = (P[rr * NA6 + cI] + P[cI * NA6 + rr]) * 0.5;
  if (is_pd6(a)) {
#pragma unroll
    for (int rr = 0; rr < NA6; ++rr)
#pragma unroll
      for (int cI = rr; cI < NA6; ++cI) {
        double v = (((P[rr * NA6 + cI] + P[cI * NA6 + rr]) + a[pk6(rr, cI)]) + a[pk6(rr, cI)]) / 4.0;
        if (bump) v = v * 2.0;
        S[rr * NA6 + cI] = v;
        S[cI * NA6 + rr] = v;
      }
    return;
  }
  double V[NA6 * NA6], w[NA6];
  jacobi6(a, V);
#pragma unroll
  for (int k = 0; k < NA6; ++k) w[k] = fabs(a[pk6(k, k)]);
#pragma unroll
  for (int rr = 0; rr < NA6; ++rr)
#pragma unroll
    for (int cI = rr; cI < NA6; ++cI) {
      double hrc = 0.0, hcr = 0.0;
#pragma unroll
      for (int k = 0; k < NA6; ++k) {
        hrc = hrc + (V[rr * NA6 + k] * w[k]) * V[cI * NA6 + k];
        hcr = hcr + (V[cI * NA6 + k] * w[k]) * V[rr * NA6 + k];
      }
      double v = (((P[rr * NA6 + cI] + P[cI * NA6 + rr]) + hrc) + hcr) / 4.0;
      if (bump) v = v * 2.0;
      S[rr * NA6 + cI] = v;
      S[cI * NA6 + rr] = v;
    }
}

// ---------------------------------------------------------------------------
// k_cell: iterEKF measurement update + EKFmatsHandler + iterMPC (lane per cell)
// ---------------------------------------------------------------------------
// row' * Sigma * row in symmetric form: T = Sigma with doubled off-diagonals,
// u_k = T_kk r_k + sum_{l>k} T_kl r_l, q = sum_k r_k u_k, explicit fma at every step
// (orc qform: 20 operations instead of the 60 of Sigma*row then row'*(.)).
__device__ __forceinline__ double qform(const double T[NPK], const double rw[NX]) {
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    double u = T[pk(k, k)] * rw[k];
#pragma unroll
    for (int l = k + 1; l < NX; ++l) u = __builtin_fma(T[pk(k, l)], rw[l], u);
    q = k == 0 ? rw[0] * u : __builtin_fma(rw[k], u, q);
  }
  return q;
}

// The plant's per-cell stores, held for the caller to issue after its last load
// (MPCEKF_PLANT_STORE_LATE): SOCn / SOCp and the advanced corner states.
struct PlantOut {
  double socn, socp;
  double x[4][6];
  int mm[4];
  bool adv[4], on;
};
__device__ __forceinline__ void plant_store(const KRom &r, const KState &s, int64_t c, int lazy_t, const PlantOut &o) {
  s.SOCn[c] = o.socn;
  s.SOCp[c] = o.socp;
  double *bx = s.bigx + (size_t)c * r.NM * 6;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!o.adv[j]) continue;
    double2 *p = reinterpret_cast<double2 *>(bx + (size_t)o.mm[j] * 6);
    p[0] = make_double2(o.x[j][0], o.x[j][1]);
    p[1] = make_double2(o.x[j][2], o.x[j][3]);
    p[2] = make_double2(o.x[j][4], o.x[j][5]);
    s.ts_plant[c * r.NM + o.mm[j]] = lazy_t;
  }
}
// OB_step's simStep (OB_step.m:188-357) for one cell at the start of k_cell's fused step:
// k_plant's arithmetic, read from the cell blob (the plant's 9 role rows are the blob's
// first C rows, D at nzp*5, diag(A) after them -- the integrator's a = 1 exactly, checked
// by build_rom -- and the res0 column after the Sigma coefficients).  Returns Vcell; the
// plant state, averages, ring inputs and timestamps are stored as k_plant stores them.
// (ring_p / po: the ring input and the state stores handed back for the caller to issue
// after its last load, MPCEKF_RING_LATE / MPCEKF_PLANT_STORE_LATE.)
template <int NZ, bool PL>
__device__ __forceinline__ double cell_plant(const KRom &r, const KState &s, const double *L, const double *tb,
                                             const double *Tp, const double *Zp, int64_t c, int lazy_t, double Iapp,
                                             double tcs, int st, double *ring_p = nullptr, PlantOut *po = nullptr) {
  constexpr int OA = NZ * NX + NZ, OR0 = NZ * NX + NZ + NX + NPK, OD = NZ * NX;
  const int stride = r.cell_stride;
  if (lazy_t) {  // this step's inputs, for the deferred updates of every model
    if (ring_p) {  // stored by the caller after its last load (MPCEKF_RING_LATE)
      *ring_p = s.priorI[c];
    } else {
      const size_t slot = (size_t)(lazy_t % LAZY_H) * s.n + c;
      s.hist_u[slot] = Iapp;
      s.hist_p[slot] = s.priorI[c];
    }
  }
  if (st & ST_ERROR) return __builtin_nan("");
  const double T = tcs + 273.15;  // OB_step.m:75
  const ETab et = etab<PL>(r, tb + r.cell_tab, T);
  double SOCnAvg = s.SOCn[c], SOCpAvg = s.SOCp[c];
  const double SOC0n = s.SOC0n[c], SOC0p = s.SOC0p[c];
  const double negSOC = SOCnAvg, posSOC = SOCpAvg;  // obs.negSOC / posSOC: pre-update (OB_step.m:226-227)
  double cellSOC = (SOCnAvg - r.th0n) / (r.th100n - r.th0n);
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (r.nZ > 1) {
    int a, b;
    two_nearest(Zp, r.nZ, cellSOC, a, b);
    iZu = a > b ? a : b; iZl = a < b ? a : b;
  }
  if (r.nT > 1) {
    int a, b;
    two_nearest(Tp, r.nT, T, a, b);
    iTu = a > b ? a : b; iTl = a < b ? a : b;
  }
  const int mm[4] = {iTl * r.nZ + iZl, iTl * r.nZ + iZu, iTu * r.nZ + iZl, iTu * r.nZ + iZu};
  double *bx = s.bigx + (size_t)c * r.NM * 6;
  // the 4 corner states as of step t-1: all loads before any store (duplicate corners)
  double xs[4][6];
  int tsj[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double2 *p = reinterpret_cast<const double2 *>(bx + (size_t)mm[j] * 6);
    const double2 q0 = p[0], q1 = p[1], q2 = p[2];
    xs[j][0] = q0.x; xs[j][1] = q0.y; xs[j][2] = q1.x; xs[j][3] = q1.y; xs[j][4] = q2.x; xs[j][5] = q2.y;
    if (lazy_t) tsj[j] = s.ts_plant[c * r.NM + mm[j]];
  }
  // the per-cell scalar chain while the corner gathers are in flight
  const double Cdleffn = et.f(0, EF_CDL, SOC0n), Cdleffp = et.f(1, EF_CDL, SOC0p);  // OB_step.m:212-219
  double dUn = et.f(0, EF_DU, SOCnAvg), dUp = et.f(1, EF_DU, SOCpAvg);
  double dQn = fabs(r.th100n - r.th0n), dQp = fabs(r.th100p - r.th0p);
  double res0n = -dQn / (3600 * r.Q - Cdleffn * dQn * dUn);
  double res0p = dQp / (3600 * r.Q - Cdleffp * dQp * dUp);
  SOCnAvg = SOCnAvg + res0n * Iapp * r.Ts;
  SOCpAvg = SOCpAvg + res0p * Iapp * r.Ts;
  if (SOCnAvg < 0) SOCnAvg = 0;
  if (SOCnAvg > 1) SOCnAvg = 1;
  if (SOCpAvg < 0) SOCpAvg = 0;
  if (SOCpAvg > 1) SOCpAvg = 1;
  if (lazy_t) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // OB_step.m:198-200 for the skipped steps, RCH inputs per round trip
      const double *a = L + mm[j] * stride + OA;
      for (int k0 = tsj[j] + 1; k0 < lazy_t; k0 += RCH) {
        double u[RCH];
        ring_chunk(s.hist_u, s, c, k0, lazy_t - 1, u);
#pragma unroll
        for (int i = 0; i < RCH; ++i)
          if (k0 + i < lazy_t) {
#pragma unroll
            for (int e = 0; e < NX; ++e) xs[j][e] = __builtin_fma(a[e], xs[j][e], u[i]);
            xs[j][NX] = __builtin_fma(1.0, xs[j][NX], u[i]);  // the integrator: a = 1
          }
      }
    }
  }
  double y[4][NPLANT];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double *B = L + mm[j] * stride;
#pragma unroll
    for (int q = 0; q < NPLANT; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < NX; ++k) acc = acc + B[q * NX + k] * xs[j][k];
      acc = acc + B[OR0 + q] * xs[j][5];
      y[j][q] = acc + B[OD + q] * Iapp;
      launder(y[j][q]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const double Zu = Zp[iZu], Zl = Zp[iZl], Tu = Tp[iTu], Tl = Tp[iTl];
  double aZ = 0.0, aT = 0.0;
  if (Zu != Zl) aZ = (cellSOC - Zl) / (Zu - Zl);
  if (Tu != Tl) aT = (T - Tl) / (Tu - Tl);
  double yk[NPLANT];
#pragma unroll
  for (int q = 0; q < NPLANT; ++q)
    yk[q] = (1 - aT) * ((1 - aZ) * y[0][q] + aZ * y[1][q]) + aT * ((1 - aZ) * y[2][q] + aZ * y[3][q]);
  double th0 = fmin(fmax(yk[R_TH0] + SOC0n, 1e-6), 1 - 1e-6);
  double th3 = fmin(fmax(yk[R_TH3] + SOC0p, 1e-6), 1 - 1e-6);
  double te1 = fmax(yk[R_TE1] + 1, 1e-6);
  double teE = fmax(yk[R_TEE] + 1, 1e-6);
  double i0n = et.f(0, EF_K0, negSOC) * sqrt(te1 * (1 - th0) * th0);  // OB_step.m:329-332
  double i0p = et.f(1, EF_K0, posSOC) * sqrt(teE * (1 - th3) * th3);
  double negEta0 = 2 * r.R * T / r.F * dasinh(yk[R_IF0] / (2 * i0n));
  double posEta3 = 2 * r.R * T / r.F * dasinh(yk[R_IF3] / (2 * i0p));
  double Uocpn0 = et.f(0, EF_U, th0), Uocpp3 = et.f(1, EF_U, th3);
  const double Rfn = et.f(0, EF_RF, negSOC), Rfp = et.f(1, EF_RF, posSOC);  // OB_step.m:339-340
  double V = posEta3 - negEta0 + yk[R_PHIE] + Uocpp3 - Uocpn0 + (Rfp * yk[R_IFDL3] - Rfn * yk[R_IFDL0]);
  V = V - r.Rc * Iapp;
  if (po) {  // the caller stores them after its last load
    po->on = true;
    po->socn = SOCnAvg;
    po->socp = SOCpAvg;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      po->mm[j] = mm[j];
      po->adv[j] = lazy_t && tsj[j] < lazy_t;
      const double *a = L + mm[j] * stride + OA;
#pragma unroll
      for (int e = 0; e < NX; ++e) po->x[j][e] = __builtin_fma(a[e], xs[j][e], Iapp);
      po->x[j][NX] = __builtin_fma(1.0, xs[j][NX], Iapp);
    }
    return V;
  }
  s.SOCn[c] = SOCnAvg;
  s.SOCp[c] = SOCpAvg;
  if (lazy_t) {  // advance the corners through step t in place
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (tsj[j] >= lazy_t) continue;
      const double *a = L + mm[j] * stride + OA;
      double2 *p = reinterpret_cast<double2 *>(bx + (size_t)mm[j] * 6);
      double x[6];
#pragma unroll
      for (int e = 0; e < NX; ++e) x[e] = __builtin_fma(a[e], xs[j][e], Iapp);
      x[NX] = __builtin_fma(1.0, xs[j][NX], Iapp);
      p[0] = make_double2(x[0], x[1]);
      p[1] = make_double2(x[2], x[3]);
      p[2] = make_double2(x[4], x[5]);
      s.ts_plant[c * r.NM + mm[j]] = lazy_t;
    }
  }
  return V;
}

// boundzk (iterEKF.m:186-205; getChatZ iterEKF.m:523-602, diagonal only) inside k_cell,
// lane per cell: for each corner j in order, its getChatV row and the 26 quadratic forms
// row' * Sigma1 * row with Sigma of the first corner (iterEKF.m:192), summed over the
// corners as ((((0 + q0) + q1) + q2) + q3) -- k_bounds' quad order, so the bits are
// k_bounds'.  Off by default: on k_cell's one-wave-per-SIMD chain the forms took as long
// as the lane-quad k_bounds at 4 waves per SIMD (r04g A/B: 2.48e8 vs 2.50e8), which also
// saved nothing by skipping the hand-off record.
#ifndef MPCEKF_CELL_BOUNDS
#define MPCEKF_CELL_BOUNDS 0
#endif
bool cell_computes_bounds() { return MPCEKF_CELL_BOUNDS != 0; }
template <int NZ>
__device__ __forceinline__ void cell_bounds(const KRom &r, const CellCtx &cc, const XI &xi, const BoundK &b, double S0,
                                            double *zo) {
  double S1b[NPK];
  load_S(cc.erec + (size_t)xi.m[0] * REC, S1b);  // the record k_cell just stored (or caught up)
#pragma unroll
  for (int k = 0; k < NX; ++k)
#pragma unroll
    for (int l = k + 1; l < NX; ++l) S1b[pk(k, l)] = 2 * S1b[pk(k, l)];
  const bool ph0pp = rowf(r, R_PHISE0, G_PPHIS);
  double ChV[4][NX], cph0[4][NX];
  const double *Cm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    Cm[j] = cc.L + xi.m[j] * cc.stride;
    chat_row(r, b.K, Cm[j], xi.g[j], ChV[j]);
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      double v = xi.g[j] * Cm[j][R_PHISE0 * NX + k];
      if (ph0pp) v = v + ChV[j][k];
      cph0[j][k] = v;
    }
  }
  // the constant-column term (c0 * S0) * c0 of each kind (C0_*), picked per row
  const double cv1 = b.C0, cv2 = b.r0n, cv3 = b.r0p, cv4 = b.dUn * b.r0n, cv5 = b.dUp * b.r0p, cv6 = -b.dUn * b.r0n;
#pragma unroll 1
  for (int q = 0; q < r.nz; ++q) {  // one form at a time
    const bool fpp = rowf(r, q, G_PPHIS), fph = rowf(r, q, G_PHIE);
    double sz = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double g = xi.g[j];
      double row[NX];
      if (fpp) {
#pragma unroll
        for (int k = 0; k < NX; ++k) row[k] = __builtin_fma(g, Cm[j][q * NX + k], ChV[j][k]);
      } else {
#pragma unroll
        for (int k = 0; k < NX; ++k) row[k] = g * Cm[j][q * NX + k];
      }
      if (fph)
#pragma unroll
        for (int k = 0; k < NX; ++k) row[k] = row[k] - cph0[j][k];
      sz = sz + qform(S1b, row);
    }
    const int kd = r.c0k[q];
    const double cv = kd == 1 ? cv1 : kd == 2 ? cv2 : kd == 3 ? cv3 : kd == 4 ? cv4 : kd == 5 ? cv5 : kd == 6 ? cv6 : 0.0;
    zo[r.perm[q]] = 3 * sqrt(sz + (cv * S0) * cv);
  }
  double sv = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) sv = sv + qform(S1b, ChV[j]);
  sv = sv + b.C0 * S0 * b.C0;
  const double rr = -r.Ts / (3600 * r.Q);
  zo[r.nz] = 3 * sqrt(sv);
  zo[r.nz + 1] = 3 * sqrt(rr * S0 * rr);
}

// 1: k_cell's simStep after the EKF's first record reads are issued, so the plant's chain
// overlaps their round trip; measured slower (r04i same-box A/B: k_cell 143 vs 134 us)
#ifndef MPCEKF_CELL_PLANT_LATE
#define MPCEKF_CELL_PLANT_LATE 0
#endif
// k_cell also runs hildreth.m (the fused step's k_hild) after a block barrier.  Off by
// default: it needs the in-kernel slow path (MPCEKF_HILD_INLINE_SLOW), and k_cell + Hildreth
// as one kernel measured 255.7 us against 161 + 89.5 as two (r04g A/B)
#ifndef MPCEKF_CELL_HILD
#define MPCEKF_CELL_HILD 0
#endif
// (with its slow lanes finished in the same kernel: MPCEKF_HILD_INLINE_SLOW)
bool cell_runs_hild() { return MPCEKF_CELL_HILD != 0 && MPCEKF_HILD_INLINE_SLOW != 0; }
__device__ __forceinline__ void hild_cell(const KCfg &cf, const KState &s, const KIO &io, int64_t c);
template <int NZ, int PARTS, bool MB = false, bool GR = false, bool PL = false>
__global__ void __launch_bounds__(256) k_cell(const KRom r, const KCfg cf, const KState s, const KIO io) {
  extern __shared__ double lds[];
  const int lo = GR ? r.cell_tab : 0;  // GR: model rows from the global blob (k_plant)
  stage_lds(lds, r.cell_blob + lo, r.cell_len - lo);
  __syncthreads();
  const double *tb = lds - lo;
  const double *Tp = tb + r.cell_tab + r.cell_tablen;
  const double *Zp = Tp + MAXT;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the plant's ring inputs for this step (MPCEKF_RING_LATE: stored after the cell's last
  // load, below, so that no load of the step waits for their stores)
  double ring_u = 0.0, ring_p = 0.0;
  bool ring_late = false;
  PlantOut pout;  // MPCEKF_PLANT_STORE_LATE: the plant's stores, issued after body
  pout.on = false;
  // the per-cell work as a lambda: its early exits return here, so every lane of the block
  // reaches the barrier of the fused Hildreth below
  auto body = [&]() {
  if (c >= s.n) return;
  const int nz = r.nz;
  const double NaN = __builtin_nan("");
  CellCtx cc;
  cc.L = GR ? r.cell_blob : lds;
  cc.Tp = Tp;
  cc.Zp = Zp;
  cc.erec = s.ekf + (size_t)c * r.NM * REC;
  cc.stride = r.cell_stride;
  const bool fplant = (PARTS & P_EKF) && !MB && io.plant;  // OB_step's simStep runs here (KRom::cell_plant)
  const double Tc = fplant && io.tc_in ? io.tc_in[c] : s.Tc[c];
  if (fplant && io.tc_in) s.Tc[c] = Tc;  // this step's TC (runMPC.m:85-92), read by every later kernel
  cc.T = Tc > 100 ? Tc : Tc + 273.15;  // iterEKF.m:62-66
  cc.et = etab<PL>(r, tb + r.cell_tab, cc.T);
  int st = s.status[c];
  const bool fused = io.mode & MODE_FUSED;
  if (io.mode & (MODE_MPC | MODE_FUSED)) s.hflag[c] = 0;  // set again only if hildreth.m must run
  STAMP(0);

  auto fail_outputs = [&]() {
    if (io.u) io.u[c] = NaN;
    if (io.v) io.v[c] = NaN;
    if (io.soc) io.soc[c] = NaN;
    if (io.phise) io.phise[c] = NaN;
    if (io.nexec) io.nexec[c] = 0;
    if (io.zk)
      for (int q = 0; q < nz + 2; ++q) io.zk[c * (nz + 2) + q] = NaN;
    if (io.zbk)
      for (int q = 0; q < nz + 2; ++q) io.zbk[c * (nz + 2) + q] = NaN;
    if (io.bnd) io.bnd[BD_M * s.n + c] = -1.0;  // no boundzk record: k_bounds leaves zbk NaN
    if (io.uk_out) io.uk_out[c] = NaN;
    if (io.x_out)
      for (int q = 0; q < 6; ++q) io.x_out[c * 6 + q] = NaN;
    if (io.junc_out) io.junc_out[c] = NaN;
    if (io.jfin_out) io.jfin_out[c] = NaN;
    if (io.normdu_out) io.normdu_out[c] = NaN;
    if (io.nviol_out) io.nviol_out[c] = 0;
    if (io.lin_out)
      for (int q = 0; q < 35; ++q) io.lin_out[c * 35 + q] = NaN;
    if (io.xm_out)
      for (int q = 0; q < 4; ++q) { io.xm_out[c * 4 + q] = -1; io.xg_out[c * 4 + q] = NaN; }
  };

  double Z[NZ];
  double xmax[NX];         // fused step: EKFmatsHandler's corner xhat, from the EKF's registers
  bool have_xmax = false;
  KR kr2{};               // the second getVariables' k0 / Rf (EKFmatsHandler reuses them)
  bool have_kr2 = false;
  double vhat = 0.0, Zsoc = 0.0;
  XI xi;
  double ik = 0.0, vk = 0.0;
  double vplant = 0.0;
  bool planted = false;
  // runMPC.m:85: [voltage, ...] = OB_step(uk, TC, cellState, ROM), first (with
  // MPCEKF_CELL_PLANT_LATE once the EKF's first record reads are issued; every path below
  // runs it before it returns)
  auto run_plant = [&]() {
    if constexpr ((PARTS & P_EKF) && !MB) {
      if (fplant && !planted) {
        if (c == 0 && io.lazy_t) *s.hslow = 0;  // k_hild_slow of the previous step has finished
        ring_u = s.uk[c];
        vplant = cell_plant<NZ, PL>(r, s, cc.L, tb, Tp, Zp, c, io.lazy_t, ring_u, Tc, st,
                                    MPCEKF_RING_LATE ? &ring_p : nullptr, MPCEKF_PLANT_STORE_LATE ? &pout : nullptr);
        ring_late = MPCEKF_RING_LATE && io.lazy_t;
        s.vk[c] = vplant;
        planted = true;
      }
    }
  };
  if (!MPCEKF_CELL_PLANT_LATE) run_plant();
  if ((PARTS & P_EKF) && (io.mode & (MODE_EKF | MODE_FUSED))) {
    if (st & ST_ERROR) {
      run_plant();
      fail_outputs();
      return;
    }
    ik = fused ? s.uk[c] : io.ik_in[c];
    vk = fused ? s.vk[c] : io.vk_in[c];  // the plant's Vcell replaces it once the plant has run
    int warn = s.warn[c];
    if (warn > cf.max_warn) {  // iterEKF.m:55-59
      run_plant();
      st |= ST_LOCKOUT | ST_ERROR;
      s.status[c] = st;
      if (fused) s.uk[c] = NaN;
      fail_outputs();
      return;
    }
    if constexpr (MB) {
    run_plant();
    // iterEKF.m:90-102 ('MB' time update), 106-108, 125-128 (gain), 160-176 (update),
    // 181-183, 199-203 (boundzk); the per-model records are never touched
    const double rs = r.Ts / (3600 * r.Q);
    const double SOC0 = s.SOC0[c];
    const double pri = s.priorI[c];
    double xm[NX], Sf[NA6 * NA6];
    {
      const double2 *p = reinterpret_cast<const double2 *>(s.mb + (size_t)c * MBREC);
      double v[MBREC];
#pragma unroll
      for (int i = 0; i < MBREC / 2; ++i) { const double2 q = p[i]; v[2 * i] = q.x; v[2 * i + 1] = q.y; }
#pragma unroll
      for (int k = 0; k < NX; ++k) xm[k] = v[k];
#pragma unroll
      for (int i = 0; i < NA6 * NA6; ++i) Sf[i] = v[6 + i];
    }
    double x0 = s.x0[c];  // xhat(end)
    get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC0 - x0 * rs, xi);  // iterEKF.m:92-93
    double amb[NA6];
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) a = a + cc.L[xi.m[j] * cc.stride + NZ * NX + NZ + k] * xi.g[j];
      amb[k] = a;
    }
    amb[NX] = 1.0;
#pragma unroll
    for (int k = 0; k < NX; ++k) xm[k] = amb[k] * xm[k] + pri;
    x0 = x0 + pri;
#pragma unroll
    for (int pp = 0; pp < NA6; ++pp)
#pragma unroll
      for (int q = 0; q < NA6; ++q) Sf[pp * NA6 + q] = (amb[pp] * Sf[pp * NA6 + q]) * amb[q] + cf.SigmaW;
    get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC0 - x0 * rs, xi);
    double xr[4][NX];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < NX; ++k) xr[j][k] = xm[k];
    vhat = get_vars<NZ>(r, cc, xi, ik, x0, SOC0, warn, st, Z, Zsoc, xr);
    if (st & ST_ERROR) {
      s.status[c] = st;
      s.warn[c] = warn;
      if (fused) s.uk[c] = NaN;
      fail_outputs();
      return;
    }
    double ChV[NA6], Lk[NA6];
    chat_mb<NZ>(r, cc, xi, SOC0 - x0 * rs, Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3], ChV);
    const double St = qform6(Sf, ChV) + cf.SigmaV;
#pragma unroll
    for (int pp = 0; pp < NA6; ++pp) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < NA6; ++k) acc = __builtin_fma(Sf[pp * NA6 + k], ChV[k], acc);
      Lk[pp] = acc / St;
    }
    const double res = vk - vhat;
#pragma unroll
    for (int k = 0; k < NX; ++k) xm[k] = __builtin_fma(Lk[k], res, xm[k]);
    x0 = __builtin_fma(Lk[NX], res, x0);
    meas_cov_mb(Sf, Lk, St, res * res > 9 * St);
    get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC0 - x0 * rs, xi);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < NX; ++k) xr[j][k] = xm[k];
    vhat = get_vars<NZ>(r, cc, xi, ik, x0, SOC0, warn, st, Z, Zsoc, xr);
    s.warn[c] = warn;
    {
      double2 *p = reinterpret_cast<double2 *>(s.mb + (size_t)c * MBREC);
      double v[MBREC];
#pragma unroll
      for (int k = 0; k < NX; ++k) v[k] = xm[k];
      v[NX] = 0.0;
#pragma unroll
      for (int i = 0; i < NA6 * NA6; ++i) v[6 + i] = Sf[i];
#pragma unroll
      for (int i = 0; i < MBREC / 2; ++i) p[i] = make_double2(v[2 * i], v[2 * i + 1]);
    }
    s.x0[c] = x0;
    if (st & ST_ERROR) {
      s.status[c] = st;
      if (fused) s.uk[c] = NaN;
      fail_outputs();
      return;
    }
    s.priorI[c] = ik;  // iterEKF.m:210
    if (io.zbk) {  // getChatZ 'MB' (iterEKF.m:537-538, 554-558, 575-576, 596-600) + iterEKF.m:199-203
      const double xSOC = SOC0 - x0 * rs;
      double ChVz[NA6];
      chat_mb<NZ>(r, cc, xi, xSOC, Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3], ChVz);
      const double res0n = -r.Ts * (cc.et.soc(0, 1) - cc.et.soc(0, 0)) / (3600 * r.Q);
      const double res0p = -r.Ts * (cc.et.soc(1, 1) - cc.et.soc(1, 0)) / (3600 * r.Q);
      const double dUn = cc.et.f(0, EF_DU, cc.et.soc(0, xSOC)), dUp = cc.et.f(1, EF_DU, cc.et.soc(1, xSOC));
      const double c0v[7] = {0.0, ChVz[NX], res0n, res0p, dUn * res0n, dUp * res0p, -dUn * res0n};
      auto chrow = [&](int q, double row[NA6]) {
#pragma unroll
        for (int k = 0; k < NX; ++k) {
          double a = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) a = a + xi.g[j] * cc.L[xi.m[j] * cc.stride + q * NX + k];
          if (rowf(r, q, G_PPHIS)) a = a + ChVz[k];
          row[k] = a;
        }
      };
      double ph0[NA6];
      chrow(R_PHISE0, ph0);
      double *zo = io.zbk + c * (nz + 2);
#pragma unroll 1
      for (int q = 0; q < nz; ++q) {
        double row[NA6];
        chrow(q, row);
        if (rowf(r, q, G_PHIE))
#pragma unroll
          for (int k = 0; k < NX; ++k) row[k] = row[k] - ph0[k];
        row[NX] = c0v[r.c0k[q]];
        zo[r.perm[q]] = 3 * sqrt(qform6(Sf, row));
      }
      zo[nz] = 3 * sqrt(qform6(Sf, ChVz));
      zo[nz + 1] = 3 * sqrt(rs * Sf[NA6 * NA6 - 1] * rs);
    }
    if (io.zk) {
#pragma unroll
      for (int q = 0; q < NZ; ++q)
        if (q < nz) io.zk[c * (nz + 2) + r.perm[q]] = Z[q];
      io.zk[c * (nz + 2) + nz] = vhat;
      io.zk[c * (nz + 2) + nz + 1] = Zsoc;
    }
    if (io.bnd) io.bnd[BD_M * s.n + c] = -1.0;  // no k_bounds record in MB
    if (io.xm_out) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { io.xm_out[c * 4 + j] = xi.m[j]; io.xg_out[c * 4 + j] = xi.g[j]; }
    }
    } else {
    double x0 = s.x0[c] + s.priorI[c];  // iterEKF.m:85-86 (models: k_bulk)
    double S0 = s.S0[c] + cf.SigmaW;
    const double SOC0 = s.SOC0[c];
    double SOC = SOC0 - x0 * (r.Ts / (3600 * r.Q));
    STAMP(1);
    get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC, xi);
    STAMP(2);
    // The 4 corner records are read once, whole (one round trip), advanced over the
    // steps their (deferred) time update skipped, used by getVariables and the gains,
    // updated and stored once; the updated xhat feeds the second getVariables and
    // EKFmatsHandler when the second getXind names the same corners.  A corner repeating
    // an earlier one (single-set-point grids) is a duplicate: the reference updates that
    // model twice in sequence, the second time from the state the first update left.
    const int t = io.lazy_t;
    bool dup[4];
    int tsj[4];
    double xr[4][NX], Sr[4][NPK];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dup[j] = false;
#pragma unroll
      for (int i = 0; i < j; ++i) dup[j] = dup[j] || xi.m[i] == xi.m[j];
      if (j < MPCEKF_REC_ONCE) load_rec(cc.erec + (size_t)xi.m[j] * REC, xr[j], Sr[j]);
      else load_x(cc.erec + (size_t)xi.m[j] * REC, xr[j]);
      tsj[j] = t ? s.ts_ekf[c * r.NM + xi.m[j]] : 0;
    }
    // step t's ring input: the plant stores this cell's priorI there (k_plant, or cell_plant
    // below, which may not have run yet)
    const double pt = t ? (fplant ? s.priorI[c] : s.hist_p[(size_t)(t % LAZY_H) * s.n + c]) : 0.0;
    run_plant();  // the records above are in flight while the plant's chain runs
    if (planted) vk = vplant;
    if (t) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (!dup[j]) replay_x(xr[j], cc.L + xi.m[j] * cc.stride + NZ * NX + NZ, tsj[j], t, pt, s, c);
#pragma unroll
      for (int j = 1; j < 4; ++j)
#pragma unroll
        for (int i = j - 1; i >= 0; --i)
          if (xi.m[i] == xi.m[j])
#pragma unroll
            for (int k = 0; k < NX; ++k) xr[j][k] = xr[i][k];
    }
    STAMP(3);
    KR kr1;
    vhat = get_vars<NZ>(r, cc, xi, ik, x0, SOC0, warn, st, Z, Zsoc, xr, 0, &kr1);
    STAMP(4);
    if (st & ST_ERROR) {
      s.status[c] = st;
      s.warn[c] = warn;
      if (fused) s.uk[c] = NaN;
      fail_outputs();
      return;
    }
    __builtin_amdgcn_sched_barrier(0);
    double ChatV[4][NX], C0;
    get_chatv<NZ>(r, cc, xi, SOC0 - x0 * (r.Ts / (3600 * r.Q)), Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3], ChatV, C0,
                  &kr1);
    if (t) replay_S(Sr[0], cc.L + xi.m[0] * cc.stride + NZ * NX + NZ, tsj[0], t, cf.SigmaW);
    double St[4], Lg[4][NX];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double row[NX];
#pragma unroll
      for (int cI = 0; cI < NX; ++cI) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) acc = __builtin_fma(Sr[0][pk(k, cI)], ChatV[j][k], acc);
        row[cI] = acc;
      }
      double acc = 0.0;
#pragma unroll
      for (int cI = 0; cI < NX; ++cI) acc = __builtin_fma(row[cI], ChatV[j][cI], acc);
      St[j] = acc + cf.SigmaV;
#pragma unroll
      for (int k = 0; k < NX; ++k) Lg[j][k] = row[k] / St[j];
    }
    double St0 = C0 * S0 * C0 + cf.SigmaV;
    double L0 = S0 * C0 / St0;
    double res = vk - vhat;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      launder(St[j]);
#pragma unroll
      for (int k = 0; k < NX; ++k) launder(Lg[j][k]);
    }
    __builtin_amdgcn_sched_barrier(0);
    STAMP(5);
    double xu[4][NX];  // corner j's xhat after its update
    // MPCEKF_S_AHEAD: corner j+1's Sigma is loaded before corner j's record is stored.  On
    // gfx950 one counter (vmcnt) covers loads and stores in issue order, so a load issued
    // after a store cannot be waited for without waiting for the store as well; loaded one
    // corner ahead, the wait for Sigma_{j+1} no longer includes corner j's store.  A corner
    // that repeats an earlier model (dup) reads its record after that store, as before.
    double Sn[NPK];
    auto s_ahead = [&](int j) {
      return MPCEKF_S_AHEAD && j < 4 && j >= MPCEKF_REC_ONCE && !dup[j];
    };
    if (s_ahead(1)) load_S(cc.erec + (size_t)xi.m[1] * REC, Sn);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double *rec = cc.erec + (size_t)xi.m[j] * REC;
      double xj[NX], Sj[NPK];
      if (dup[j]) {
        load_rec(rec, xj, Sj);  // as the earlier update of this model left it
      } else {
#pragma unroll
        for (int k = 0; k < NX; ++k) xj[k] = xr[j][k];
        if (j < MPCEKF_REC_ONCE) {
#pragma unroll
          for (int k = 0; k < NPK; ++k) Sj[k] = Sr[j][k];
        } else if (s_ahead(j)) {
#pragma unroll
          for (int k = 0; k < NPK; ++k) Sj[k] = Sn[k];
        } else {
          load_S(rec, Sj);
        }
        if (t && j > 0) replay_S(Sj, cc.L + xi.m[j] * cc.stride + NZ * NX + NZ, tsj[j], t, cf.SigmaW);
      }
      meas_update_regs<MPCEKF_CELL_OUTLINE>(xj, Sj, Lg[j], St[j], res);
      if (j + 1 < 4 && s_ahead(j + 1)) load_S(cc.erec + (size_t)xi.m[j + 1] * REC, Sn);
      store_rec(rec, xj, Sj);
      if (t) s.ts_ekf[c * r.NM + xi.m[j]] = t;
#pragma unroll
      for (int k = 0; k < NX; ++k) xu[j][k] = xj[k];
      __builtin_amdgcn_sched_barrier(0);
    }
    STAMP(6);
    x0 = __builtin_fma(L0, res, x0);
    S0 = S0 - L0 * St0 * L0;
    SOC = SOC0 - x0 * (r.Ts / (3600 * r.Q));
    int m1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m1[j] = xi.m[j];
    get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC, xi);
    // same corners: their xhat is in registers and current; else catch the new corners
    // up and read them (their records are the stored ones)
    const bool same = m1[0] == xi.m[0] && m1[1] == xi.m[1] && m1[2] == xi.m[2] && m1[3] == xi.m[3] &&
                      !(dup[1] || dup[2] || dup[3]);
    if (!same) {
      if (io.lazy_t) ekf_catch_up4<NZ>(s, cc, r.NM, xi.m, c, io.lazy_t, cf.SigmaW, pt);
#pragma unroll
      for (int j = 0; j < 4; ++j) load_x(cc.erec + (size_t)xi.m[j] * REC, xu[j]);
    }
    STAMP(7);
    vhat = get_vars<NZ>(r, cc, xi, ik, x0, SOC0, warn, st, Z, Zsoc, xu, 0, &kr2);
    have_kr2 = true;
    const int jm = corner_max(xi);
#pragma unroll
    for (int k = 0; k < NX; ++k) xmax[k] = jm == 0 ? xu[0][k] : jm == 1 ? xu[1][k] : jm == 2 ? xu[2][k] : xu[3][k];
    have_xmax = true;
    __builtin_amdgcn_sched_barrier(0);
    STAMP(8);
    s.warn[c] = warn;
    if (st & ST_ERROR) {
      s.status[c] = st;
      s.x0[c] = x0;
      s.S0[c] = S0;
      if (fused) s.uk[c] = NaN;
      fail_outputs();
      return;
    }
    if (io.bnd) {  // boundzk (iterEKF.m:186-205) runs in k_bounds from this record
      double *bd = io.bnd;
      const int64_t n = s.n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bd[(BD_G + j) * n + c] = xi.g[j];
        bd[(BD_M + j) * n + c] = xi.m[j];
      }
      const BoundK b =
          bound_k(r, cc, SOC0 - x0 * (r.Ts / (3600 * r.Q)), Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3], &kr2);
#pragma unroll
      for (int i = 0; i < 11; ++i) bd[(BD_K + i) * n + c] = bound_field(b, i);
      bd[BD_S0 * n + c] = S0;
    }
    STAMP(9);
    s.x0[c] = x0;
    s.S0[c] = S0;
    s.priorI[c] = ik;  // iterEKF.m:210
    if (io.zk) {
#pragma unroll
      for (int q = 0; q < NZ; ++q)
        if (q < nz) io.zk[c * (nz + 2) + r.perm[q]] = Z[q];
      io.zk[c * (nz + 2) + nz] = vhat;
      io.zk[c * (nz + 2) + nz + 1] = Zsoc;
    }
    if (io.xm_out) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { io.xm_out[c * 4 + j] = xi.m[j]; io.xg_out[c * 4 + j] = xi.g[j]; }
    }
    if (MPCEKF_CELL_BOUNDS && io.zbk && !io.bnd)
      cell_bounds<NZ>(r, cc, xi, bound_k(r, cc, SOC0 - x0 * (r.Ts / (3600 * r.Q)), Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3]),
                      S0, io.zbk + c * (nz + 2));
    }  // OB
  }
  if (!(PARTS & (P_MPC | P_LIN))) return;
  // The fused step's second kernel: cells the iterEKF kernel failed are finished.
  if (!(PARTS & P_EKF) && fused) {
    if (st & ST_ERROR) return;
    vk = s.vk[c];
  }

  Lin L;
  if (io.mode & (MODE_LIN | MODE_FUSED)) {
    double zr[NROLE];
    if (fused && (PARTS & P_EKF)) {
#pragma unroll
      for (int q = 0; q < NROLE; ++q) zr[q] = Z[q];
    } else {
      if (!fused && (st & ST_ERROR)) { fail_outputs(); return; }
#pragma unroll
      for (int q = 0; q < NROLE; ++q) zr[q] = io.zk_in[c * (nz + 2) + r.perm[q]];
      Zsoc = io.zk_in[c * (nz + 2) + nz + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) { xi.m[j] = io.xm_in[c * 4 + j]; xi.g[j] = io.xg_in[c * 4 + j]; }
    }
    mats_handler<NZ>(r, cc, xi, zr, Zsoc, Tc + 273.15, L, MB ? s.x0[c] : 0.0, xmax, fused && (PARTS & P_EKF) && have_xmax,
                     fused && (PARTS & P_EKF) && have_kr2 ? &kr2 : nullptr);
    if (io.lin_out) lin_store(io.lin_out + c * 35, L);
    if (io.x_out)
#pragma unroll
      for (int q = 0; q < 6; ++q) io.x_out[c * 6 + q] = L.xhat[q];  // x_store (runMPC.m:108)
  }
  STAMP(10);
  if (PARTS & P_LIN) {  // iterMPC runs in the wide-horizon kernels (mpcekf_wide.hip) from lin_out / zsoc_out
    if (fused) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) acc = acc + L.Cphi[k] * L.xhat[k];
      if (io.phise) io.phise[c] = acc + s.uk[c] * L.Dphi + L.bphi;  // runMPC.m:94-95
      if (io.v) io.v[c] = vk;
      if (io.soc) io.soc[c] = Zsoc;
      if (io.zsoc_out) io.zsoc_out[c] = Zsoc;
    }
    return;
  }

#ifndef PROBE_NO_MPC
  if (io.mode & (MODE_MPC | MODE_FUSED)) {
    if (!fused) {
      if (st & ST_ERROR) { fail_outputs(); return; }
      lin_load(io.lin_in + c * 35, L);
      Zsoc = io.soc_k1_in[c];
    }
    double uk_1 = s.uk_1[c];
    double ukin = fused ? s.uk[c] : 0.0;
    double phise = 0.0;
    if (fused) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) acc = acc + L.Cphi[k] * L.xhat[k];
      phise = acc + ukin * L.Dphi + L.bphi;  // runMPC.m:94-95
    }
    MpcOut o;
    MpcSetup Pm;
    bool need = mpc_setup(cf, L, uk_1, Zsoc, Pm, o);
    if (fused) {
      if (io.v) io.v[c] = vk;
      if (io.soc) io.soc[c] = Zsoc;
      if (io.phise) io.phise[c] = phise;
    }
    if (s.J_unc) s.J_unc[c] = o.J_unc;
    if (io.junc_out) io.junc_out[c] = o.J_unc;
    STAMP(11);
    s.hflag[c] = need ? 1 : 0;
    if (need) {  // hildreth.m runs in k_hild
      double *pb = s.prob;
      const int64_t n = s.n;
#pragma unroll
      for (int a = 0; a < NC; ++a) {
        pb[(PB_F + a) * n + c] = Pm.F[a];
#pragma unroll
        for (int b = 0; b < NC; ++b) pb[(PB_E + a * NC + b) * n + c] = Pm.E[a][b];
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        pb[(PB_HV + i) * n + c] = Pm.Cn.Hv[i];
        pb[(PB_HE + i) * n + c] = Pm.Cn.He[i];
        pb[(PB_HS + i) * n + c] = Pm.Cn.Hs[i];
        pb[(PB_ERR + i) * n + c] = Pm.e[i];
      }
#pragma unroll
      for (int i = 0; i < NCON; ++i) pb[(PB_GAM + i) * n + c] = Pm.Cn.gam[i];
      pb[PB_RU * n + c] = Pm.Ru;
      pb[PB_UK1 * n + c] = uk_1;
    } else {
      o.nexec = 0;
      mpc_finish(Pm.Cn, Pm.e, Pm.Ru, Pm.DU, uk_1, o);
      s.uk_1[c] = uk_1;
      if (s.J_fin) { s.J_fin[c] = o.J_fin; s.nviol[c] = o.nviol; }
      cost_out(io, c, o.J_fin, o.nviol, norm_du<NC>(Pm.DU));
      if (io.uk_out) io.uk_out[c] = o.uk;
      if (io.nexec) io.nexec[c] = 0;
      if (fused) {
        s.uk[c] = o.uk;
        if (io.u) io.u[c] = o.uk;
      }
    }
  }
#endif
  };
  body();
  if (MPCEKF_PLANT_STORE_LATE && pout.on) plant_store(r, s, c, io.lazy_t, pout);
  if (ring_late) {  // every path of body ran the plant; the ring's slot t is read by no load of this step
    const size_t slot = (size_t)(io.lazy_t % LAZY_H) * s.n + c;
    s.hist_u[slot] = ring_u;
    s.hist_p[slot] = ring_p;
  }
  if constexpr (MPCEKF_CELL_HILD && (PARTS & P_MPC) != 0) {
    if (io.hild) {  // hildreth.m in the same kernel (no k_hild launch): the blob's LDS becomes the
      __syncthreads();  // per-lane Hildreth slots once every wave of the block is done with it
      if (c < s.n) hild_cell(cf, s, io, c);
    }
  }
}

// OB_step's simStep (OB_step.m:188-357) at the start of k_ekf4's fused step: k_plant4's lane
// quad (lane j = corner j: its gather, replay and 9 output rows; the blend by quad
// broadcasts in the one-lane order; the per-cell scalar chain the same in all four lanes)
// on cell_plant's cell-blob layout.  Every live lane stores the per-cell values (the same
// bits), so each lane's later reads of them (the ring slot of this step) follow its own
// store.  Returns Vcell in every lane of the quad; k_plant / cell_plant's bits.
template <int NZ, bool PL>
__device__ __forceinline__ double quad_plant(const KRom &r, const KState &s, const double *L, const double *tb,
                                             const double *Tp, const double *Zp, int64_t c, int j, bool live,
                                             int lazy_t, double Iapp, double tcs, int st) {
  constexpr int OA = NZ * NX + NZ, OR0 = NZ * NX + NZ + NX + NPK, OD = NZ * NX;
  const int stride = r.cell_stride;
  if (lazy_t && live) {  // this step's inputs, for the deferred updates of every model
    const size_t slot = (size_t)(lazy_t % LAZY_H) * s.n + c;
    s.hist_u[slot] = Iapp;
    s.hist_p[slot] = s.priorI[c];
  }
  if (st & ST_ERROR) return __builtin_nan("");
  const double T = tcs + 273.15;  // OB_step.m:75
  const ETab et = etab<PL>(r, tb + r.cell_tab, T);
  double SOCnAvg = s.SOCn[c], SOCpAvg = s.SOCp[c];
  const double SOC0n = s.SOC0n[c], SOC0p = s.SOC0p[c];
  const double negSOC = SOCnAvg, posSOC = SOCpAvg;  // obs.negSOC / posSOC: pre-update (OB_step.m:226-227)
  double cellSOC = (SOCnAvg - r.th0n) / (r.th100n - r.th0n);
  int iZu = 0, iZl = 0, iTu = 0, iTl = 0;
  if (r.nZ > 1) {
    int a, b;
    two_nearest(Zp, r.nZ, cellSOC, a, b);
    iZu = a > b ? a : b; iZl = a < b ? a : b;
  }
  if (r.nT > 1) {
    int a, b;
    two_nearest(Tp, r.nT, T, a, b);
    iTu = a > b ? a : b; iTl = a < b ? a : b;
  }
  // this lane's corner: mm = {Tl Zl, Tl Zu, Tu Zl, Tu Zu}[j]
  const int mj = ((j & 2) ? iTu : iTl) * r.nZ + ((j & 1) ? iZu : iZl);
  double *bx = s.bigx + ((size_t)c * r.NM + mj) * 6;
  double xs[6];
  {
    const double2 *p = reinterpret_cast<const double2 *>(bx);
    const double2 q0 = p[0], q1 = p[1], q2 = p[2];
    xs[0] = q0.x; xs[1] = q0.y; xs[2] = q1.x; xs[3] = q1.y; xs[4] = q2.x; xs[5] = q2.y;
  }
  const int tsj = lazy_t ? s.ts_plant[c * r.NM + mj] : 0;
  const double Cdleffn = et.f(0, EF_CDL, SOC0n), Cdleffp = et.f(1, EF_CDL, SOC0p);  // OB_step.m:212-219
  double dUn = et.f(0, EF_DU, SOCnAvg), dUp = et.f(1, EF_DU, SOCpAvg);
  double dQn = fabs(r.th100n - r.th0n), dQp = fabs(r.th100p - r.th0p);
  double res0n = -dQn / (3600 * r.Q - Cdleffn * dQn * dUn);
  double res0p = dQp / (3600 * r.Q - Cdleffp * dQp * dUp);
  SOCnAvg = SOCnAvg + res0n * Iapp * r.Ts;
  SOCpAvg = SOCpAvg + res0p * Iapp * r.Ts;
  if (SOCnAvg < 0) SOCnAvg = 0;
  if (SOCnAvg > 1) SOCnAvg = 1;
  if (SOCpAvg < 0) SOCpAvg = 0;
  if (SOCpAvg > 1) SOCpAvg = 1;
  const double Zu = Zp[iZu], Zl = Zp[iZl], Tu = Tp[iTu], Tl = Tp[iTl];
  double aZ = 0.0, aT = 0.0;
  if (Zu != Zl) aZ = (cellSOC - Zl) / (Zu - Zl);
  if (Tu != Tl) aT = (T - Tl) / (Tu - Tl);
  const double *a = L + mj * stride + OA;
  if (lazy_t)  // OB_step.m:198-200 for the skipped steps, RCH ring inputs per round trip
    for (int k0 = tsj + 1; k0 < lazy_t; k0 += RCH) {
      double u[RCH];
      ring_chunk(s.hist_u, s, c, k0, lazy_t - 1, u);
#pragma unroll
      for (int i = 0; i < RCH; ++i)
        if (k0 + i < lazy_t) {
#pragma unroll
          for (int e = 0; e < NX; ++e) xs[e] = __builtin_fma(a[e], xs[e], u[i]);
          xs[NX] = __builtin_fma(1.0, xs[NX], u[i]);  // the integrator: a = 1
        }
    }
  const double *B = L + mj * stride;
  double yk[NPLANT];
#pragma unroll
  for (int q = 0; q < NPLANT; ++q) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k) acc = acc + B[q * NX + k] * xs[k];
    acc = acc + B[OR0 + q] * xs[5];
    const double y = acc + B[OD + q] * Iapp;
    const double y0 = qbc<0>(y), y1 = qbc<1>(y), y2 = qbc<2>(y), y3 = qbc<3>(y);
    yk[q] = (1 - aT) * ((1 - aZ) * y0 + aZ * y1) + aT * ((1 - aZ) * y2 + aZ * y3);
  }
  double th0 = fmin(fmax(yk[R_TH0] + SOC0n, 1e-6), 1 - 1e-6);
  double th3 = fmin(fmax(yk[R_TH3] + SOC0p, 1e-6), 1 - 1e-6);
  double te1 = fmax(yk[R_TE1] + 1, 1e-6);
  double teE = fmax(yk[R_TEE] + 1, 1e-6);
  double i0n = et.f(0, EF_K0, negSOC) * sqrt(te1 * (1 - th0) * th0);  // OB_step.m:329-332
  double i0p = et.f(1, EF_K0, posSOC) * sqrt(teE * (1 - th3) * th3);
  double negEta0 = 2 * r.R * T / r.F * dasinh(yk[R_IF0] / (2 * i0n));
  double posEta3 = 2 * r.R * T / r.F * dasinh(yk[R_IF3] / (2 * i0p));
  double Uocpn0 = et.f(0, EF_U, th0), Uocpp3 = et.f(1, EF_U, th3);
  const double Rfn = et.f(0, EF_RF, negSOC), Rfp = et.f(1, EF_RF, posSOC);  // OB_step.m:339-340
  double V = posEta3 - negEta0 + yk[R_PHIE] + Uocpp3 - Uocpn0 + (Rfp * yk[R_IFDL3] - Rfn * yk[R_IFDL0]);
  V = V - r.Rc * Iapp;
  if (live) {
    s.SOCn[c] = SOCnAvg;
    s.SOCp[c] = SOCpAvg;
  }
  if (live && lazy_t && tsj < lazy_t) {  // advance this corner through step t in place
    double2 *p = reinterpret_cast<double2 *>(bx);
    double x[6];
#pragma unroll
    for (int e = 0; e < NX; ++e) x[e] = __builtin_fma(a[e], xs[e], Iapp);
    x[NX] = __builtin_fma(1.0, xs[NX], Iapp);
    p[0] = make_double2(x[0], x[1]);
    p[1] = make_double2(x[2], x[3]);
    p[2] = make_double2(x[4], x[5]);
    s.ts_plant[c * r.NM + mj] = lazy_t;
  }
  return V;
}

// ---------------------------------------------------------------------------
// k_ekf4: the fused step's iterEKF ('OB', iterEKF.m:55-210) with a lane quad per cell,
// lane j = corner j of getXind: its record's catch-up, its getVariables term, its
// getChatV row, gain and measurement update run in parallel; the corner sums keep the
// one-lane order through DPP broadcasts (get_vars<NZ, true>), so every result is
// k_cell's to the bit.  EKFmatsHandler + iterMPC follow in k_cell<NZ, P_MPC> from the
// zk / Xind hand-off.  Needs distinct corners (nT > 1 and nZ > 1; host checks).
// 1024-thread blocks (256 cells): the ~130 KB ROM blob is staged once per CU and the
// CU runs 4 waves per SIMD.
// ---------------------------------------------------------------------------
template <int NZ, int BLOCK, bool GR, bool PL>
__global__ void __launch_bounds__(BLOCK) k_ekf4(const KRom r, const KCfg cf, const KState s, const KIO io) {
  extern __shared__ double lds[];
  const int lo = GR ? r.cell_tab : 0;  // GR: model rows from the global blob (k_plant)
  stage_lds(lds, r.cell_blob + lo, r.cell_len - lo);
  __syncthreads();
  const double *tb = lds - lo;
  const double *Tp = tb + r.cell_tab + r.cell_tablen;
  const double *Zp = Tp + MAXT;
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  const int j = (int)(gt & 3);
  const int64_t cq = gt >> 2;
  const bool live = cq < n;
  const int64_t c = live ? cq : n - 1;  // lanes past n ride along (quad exchanges), write nothing
  const int nz = r.nz;
  const double NaN = __builtin_nan("");
  CellCtx cc;
  cc.L = GR ? r.cell_blob : lds;
  cc.Tp = Tp;
  cc.Zp = Zp;
  cc.erec = s.ekf + (size_t)c * r.NM * REC;
  cc.stride = r.cell_stride;
  const bool fplant = io.plant;  // OB_step's simStep runs here (KRom::cell_plant; k_cell's fplant)
  const double Tc = fplant && io.tc_in ? io.tc_in[c] : s.Tc[c];
  if (fplant && io.tc_in && live && j == 0) s.Tc[c] = Tc;  // this step's TC (runMPC.m:85-92)
  cc.T = Tc > 100 ? Tc : Tc + 273.15;  // iterEKF.m:62-66
  cc.et = etab<PL>(r, tb + r.cell_tab, cc.T);
  int st = s.status[c];
  const int t = io.lazy_t;
  if (live && j == 0) s.hflag[c] = 0;
  // runMPC.m:85: [voltage, ...] = OB_step(uk, TC, cellState, ROM) first
  double vplant = 0.0;
  if (fplant) {
    if (gt == 0 && t) *s.hslow = 0;  // k_hild_slow of the previous step has finished
    vplant = quad_plant<NZ, PL>(r, s, cc.L, tb, Tp, Zp, c, j, live, t, s.uk[c], Tc, st);
    if (live && j == 0) s.vk[c] = vplant;
  }
  auto fail_outputs = [&]() {
    if (!live) return;
    if (j == 0) {
      if (io.u) io.u[c] = NaN;
      if (io.v) io.v[c] = NaN;
      if (io.soc) io.soc[c] = NaN;
      if (io.phise) io.phise[c] = NaN;
      if (io.nexec) io.nexec[c] = 0;
      if (io.bnd) io.bnd[BD_M * n + c] = -1.0;
      if (io.x_out)
        for (int q = 0; q < 6; ++q) io.x_out[c * 6 + q] = NaN;
      if (io.junc_out) io.junc_out[c] = NaN;
      if (io.jfin_out) io.jfin_out[c] = NaN;
      if (io.normdu_out) io.normdu_out[c] = NaN;
      if (io.nviol_out) io.nviol_out[c] = 0;
    }
    if (io.zk)
      for (int q = j; q < nz + 2; q += 4) io.zk[c * (nz + 2) + q] = NaN;
    if (io.zbk)
      for (int q = j; q < nz + 2; q += 4) io.zbk[c * (nz + 2) + q] = NaN;
    if (io.xm_out) { io.xm_out[c * 4 + j] = -1; io.xg_out[c * 4 + j] = NaN; }
  };
  if (st & ST_ERROR) {
    fail_outputs();
    return;
  }
  const double ik = s.uk[c], vk = fplant ? vplant : s.vk[c];
  int warn = s.warn[c];
  if (warn > cf.max_warn) {  // iterEKF.m:55-59
    st |= ST_LOCKOUT | ST_ERROR;
    if (live && j == 0) { s.status[c] = st; s.uk[c] = NaN; }
    fail_outputs();
    return;
  }
  double x0 = s.x0[c] + s.priorI[c];  // iterEKF.m:85-86
  double S0 = s.S0[c] + cf.SigmaW;
  const double SOC0 = s.SOC0[c];
  XI xi;
  get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC0 - x0 * (r.Ts / (3600 * r.Q)), xi);
  // this lane's corner: record, caught up over the steps its time update skipped
  const int mj = xi.m[j];
  double *rec = cc.erec + (size_t)mj * REC;
  const double *am = cc.L + mj * cc.stride + NZ * NX + NZ;  // diag(A), then a_p a_q
  double xr[1][NX];
  load_x(rec, xr[0]);
  const int tsj = s.ts_ekf[c * r.NM + mj];
  const double pt = s.hist_p[(size_t)(t % LAZY_H) * n + c];
  replay_x(xr[0], am, tsj, t, pt, s, c);
  __builtin_amdgcn_sched_barrier(0);
  double Z[NZ], Zsoc;
  double vhat = get_vars<NZ, true>(r, cc, xi, ik, x0, SOC0, warn, st, Z, Zsoc, xr, j);
  if (st & ST_ERROR) {
    if (live && j == 0) { s.status[c] = st; s.warn[c] = warn; s.uk[c] = NaN; }
    fail_outputs();
    return;
  }
  __builtin_amdgcn_sched_barrier(0);
  // getChatV (iterEKF.m:421-519): this corner's row; gains against corner 1's Sigma
  const ChatK K = chat_k(r, cc, SOC0 - x0 * (r.Ts / (3600 * r.Q)), Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3]);
  double Ch[NX];
  chat_row(r, K, cc.L + mj * cc.stride, xi.g[j], Ch);
  const double C0 = chat0(r, K);
  double Sj[NPK];
  load_S(rec, Sj);
  replay_S(Sj, am, tsj, t, cf.SigmaW);
  double S1[NPK];
#pragma unroll
  for (int i = 0; i < NPK; ++i) S1[i] = qbc<0>(Sj[i]);
  double row[NX];
#pragma unroll
  for (int cI = 0; cI < NX; ++cI) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k) acc = __builtin_fma(S1[pk(k, cI)], Ch[k], acc);
    row[cI] = acc;
  }
  double acc = 0.0;
#pragma unroll
  for (int cI = 0; cI < NX; ++cI) acc = __builtin_fma(row[cI], Ch[cI], acc);
  const double Stj = acc + cf.SigmaV;
  double Lg[NX];
#pragma unroll
  for (int k = 0; k < NX; ++k) Lg[k] = row[k] / Stj;
  const double St0 = C0 * S0 * C0 + cf.SigmaV;
  const double L0 = S0 * C0 / St0;
  const double res = vk - vhat;
  __builtin_amdgcn_sched_barrier(0);
  // iterEKF.m:137-153: corner j's record (distinct corners: the updates are independent)
  meas_update_regs<true>(xr[0], Sj, Lg, Stj, res);
  if (live) {
    store_rec(rec, xr[0], Sj);
    s.ts_ekf[c * r.NM + mj] = t;
  }
  __builtin_amdgcn_sched_barrier(0);
  x0 = __builtin_fma(L0, res, x0);
  S0 = S0 - L0 * St0 * L0;
  int mold[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) mold[i] = xi.m[i];
  get_xind(r.nT, r.nZ, Tp, Zp, cc.T, SOC0 - x0 * (r.Ts / (3600 * r.Q)), xi);
  // the new corner j: one this step just updated (its state comes from that lane's
  // registers), or an untouched model whose record is caught up to step t here
  // (ekf_catch_up4)
  const int mn = xi.m[j];
  int src = -1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (mold[i] == mn) src = i;
  {
    const int from = (threadIdx.x & ~3) + (src < 0 ? j : src);
#pragma unroll
    for (int k = 0; k < NX; ++k) xr[0][k] = shfl64(xr[0][k], from);
  }
  if (src < 0) {
    double *recn = cc.erec + (size_t)mn * REC;
    const int tsn = s.ts_ekf[c * r.NM + mn];
    double Sn[NPK];
    load_rec(recn, xr[0], Sn);
    if (tsn < t) {
      const double *an = cc.L + mn * cc.stride + NZ * NX + NZ;
      replay_x(xr[0], an, tsn, t, pt, s, c);
      replay_S(Sn, an, tsn, t, cf.SigmaW);
      if (live) {
        store_rec(recn, xr[0], Sn);
        s.ts_ekf[c * r.NM + mn] = t;
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  vhat = get_vars<NZ, true>(r, cc, xi, ik, x0, SOC0, warn, st, Z, Zsoc, xr, j);
  __builtin_amdgcn_sched_barrier(0);
  if (!live) return;
  if (j == 0) s.warn[c] = warn;
  if (st & ST_ERROR) {
    if (j == 0) { s.status[c] = st; s.x0[c] = x0; s.S0[c] = S0; s.uk[c] = NaN; }
    fail_outputs();
    return;
  }
  if (io.bnd) {  // boundzk (iterEKF.m:186-205) runs in k_bounds from this record
    io.bnd[(BD_G + j) * n + c] = xi.g[j];
    io.bnd[(BD_M + j) * n + c] = xi.m[j];
    const BoundK b = bound_k(r, cc, SOC0 - x0 * (r.Ts / (3600 * r.Q)), Z[R_TE1], Z[R_TH0], Z[R_TEE], Z[R_TH3]);
#pragma unroll
    for (int i = 0; i < 11; ++i)
      if ((i & 3) == j) io.bnd[(BD_K + i) * n + c] = bound_field(b, i);
    if (j == 3) io.bnd[BD_S0 * n + c] = S0;
  }
  if (j == 0) {
    s.x0[c] = x0;
    s.S0[c] = S0;
    s.priorI[c] = ik;  // iterEKF.m:210
  }
  if (io.zk) {
#pragma unroll
    for (int q = 0; q < NZ; ++q)
      if (q < nz && (q & 3) == j) io.zk[c * (nz + 2) + r.perm[q]] = Z[q];
    if (j == 1) io.zk[c * (nz + 2) + nz] = vhat;
    if (j == 2) io.zk[c * (nz + 2) + nz + 1] = Zsoc;
  }
  if (io.xm_out) { io.xm_out[c * 4 + j] = xi.m[j]; io.xg_out[c * 4 + j] = xi.g[j]; }
}

// ---------------------------------------------------------------------------
// k_bounds: boundzk (iterEKF.m:186-205; getChatZ iterEKF.m:523-602), diagonal only.
// A lane quad per cell, lane j = corner j: its getChatV row, its 26 quadratic forms
// row' * Sigma1 * row; the corner sums keep k_cell's order ((((0 + q0) + q1) + q2)
// + q3) through DPP broadcasts, so the result is the one-lane form's bits.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double quad_sum_seq(double v) {  // (((0 + v0) + v1) + v2) + v3
  return (((0.0 + qbc<0>(v)) + qbc<1>(v)) + qbc<2>(v)) + qbc<3>(v);
}

// 256 cells per block: the ~90 KB model blob leaves room for one block per CU, so the
// block is the CU's whole occupancy (4 waves per SIMD) and stages the blob once.
constexpr int BOUNDS_BLOCK = 1024;
// k_bounds stages only the models of the cell blob (its getChatV scalars come from k_cell)
__host__ __device__ inline int bounds_c0_base(const KRom &r) { return r.rom_global ? 0 : r.cell_tab + 1; }
template <int NZ, bool GR>
__global__ void __launch_bounds__(BOUNDS_BLOCK) k_bounds(const KRom r, const KState s, const double *bd, double *zbk) {
  extern __shared__ double lds[];
  if (!GR) stage_lds(lds, r.cell_blob, r.cell_tab);  // GR: model rows from the global blob
  __syncthreads();
  const double *L = GR ? r.cell_blob : lds;
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  const int j = (int)(gt & 3);
  const int64_t cq = gt >> 2;
  const int64_t c = cq < n ? cq : n - 1;  // lanes past n ride along (quad exchanges)
  const int nz = r.nz;
  const bool valid = cq < n && bd[BD_M * n + c] >= 0.0;
  const double g = bd[(BD_G + j) * n + c];
  const int m = valid ? (int)bd[(BD_M + j) * n + c] : 0;
  const double *Cm = L + m * r.cell_stride;
  const double S0 = bd[BD_S0 * n + c];
  // SigmaX of the first corner for all four (iterEKF.m:191)
  double S1b[NPK];
  load_S(s.ekf + ((size_t)c * r.NM + (valid ? (int)bd[BD_M * n + c] : 0)) * REC, S1b);
#pragma unroll
  for (int k = 0; k < NX; ++k)
#pragma unroll
    for (int l = k + 1; l < NX; ++l) S1b[pk(k, l)] = 2 * S1b[pk(k, l)];
  // getChatV's scalars at the updated state, from k_cell (bound_k)
  ChatK K;
  K.Rfn = bd[(BD_K + 0) * n + c];
  K.Rfp = bd[(BD_K + 1) * n + c];
  K.Rctn = bd[(BD_K + 2) * n + c];
  K.Rctp = bd[(BD_K + 3) * n + c];
  K.dUn0 = bd[(BD_K + 4) * n + c];
  K.dUp3 = bd[(BD_K + 5) * n + c];
  double ChV[NX];
  chat_row(r, K, Cm, g, ChV);
  const double ChV0 = bd[BD_C0 * n + c];
  const double res0n = bd[BD_R0N * n + c], res0p = bd[BD_R0P * n + c];
  const double dUn = bd[BD_DUN * n + c], dUp = bd[BD_DUP * n + c];
  const bool ph0pp = rowf(r, R_PHISE0, G_PPHIS);
  double cph0[NX];
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    double v = g * Cm[R_PHISE0 * NX + k];
    if (ph0pp) v = v + ChV[k];
    cph0[k] = v;
  }
  // The constant-column terms (c0 * S0) * c0 of the 7 kinds (C0_*) in an LDS row per
  // cell, lane j filling kinds j and j + 4: each form then adds its term by a uniform
  // offset instead of a select chain.
  double *c0t = lds + (GR ? 0 : r.cell_tab + 1) + (threadIdx.x >> 2) * 8;
  {
    const double cv[8] = {0.0, ChV0, res0n, res0p, dUn * res0n, dUp * res0p, -dUn * res0n, 0.0};
    double lo = cv[0], hi = cv[4];
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (j == i) { lo = cv[i]; hi = cv[i + 4]; }
    c0t[j] = (lo * S0) * lo;
    c0t[j + 4] = (hi * S0) * hi;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // Forms q = j, j + 4, ... are this lane's to finish: their sums and output slots.
  constexpr int NOWN = (NZ + 3) / 4;
  double mine[NOWN];
  int slot[NOWN];
#pragma unroll
  for (int i = 0; i < NOWN; ++i) { mine[i] = 0.0; slot[i] = -1; }
#pragma unroll
  for (int q = 0; q < NZ; ++q) {
    double row[NX];
    const bool fpp = rowf(r, q, G_PPHIS), fph = rowf(r, q, G_PHIE);
    // uniform branches (the empty volatile asm keeps them from being if-converted)
    if (fpp) {
      asm volatile("");
#pragma unroll
      for (int k = 0; k < NX; ++k) row[k] = __builtin_fma(g, Cm[q * NX + k], ChV[k]);
    } else {
      asm volatile("");
#pragma unroll
      for (int k = 0; k < NX; ++k) row[k] = g * Cm[q * NX + k];
    }
    if (fph) {
      asm volatile("");
#pragma unroll
      for (int k = 0; k < NX; ++k) row[k] = row[k] - cph0[k];
    }
    const double qf = qform(S1b, row);
    const double sz = quad_sum_seq(qf) + c0t[r.c0k[q]];
    if ((q & 3) == j && q < nz) {
      mine[q >> 2] = sz;
      slot[q >> 2] = r.perm[q];
    }
    __builtin_amdgcn_sched_barrier(0);  // one form at a time: 128 VGPRs at 4 waves/SIMD
  }
  double *zo = zbk + c * (nz + 2);
#pragma unroll
  for (int i = 0; i < NOWN; ++i)
    if (valid && slot[i] >= 0) zo[slot[i]] = 3 * sqrt(mine[i]);
  const double acc = qform(S1b, ChV);
  double SigV = quad_sum_seq(acc);
  SigV = SigV + ChV0 * S0 * ChV0;
  const double rr = -r.Ts / (3600 * r.Q);
  const double SigSOC = rr * S0 * rr;
  if (valid && j == 0) {
    zo[nz] = 3 * sqrt(SigV);
    zo[nz + 1] = 3 * sqrt(SigSOC);
  }
}

// ---------------------------------------------------------------------------
// k_hild: hildreth.m + iterMPC.m:68-95 for the cells k_cell flagged
// ---------------------------------------------------------------------------
// The QP record of cell c (PB_*) -> Cons, E and K = M*(E\F) + gamma (hildreth.m:29).
__device__ __forceinline__ void hild_load(const KState &s, int64_t c, Cons &Cn, double E[NC][NC], double K[NCON]) {
  const int64_t n = s.n;
  const double *pb = s.prob;
  double F[NC], y[NC], R[NC][NC];
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    F[a] = pb[(PB_F + a) * n + c];
#pragma unroll
    for (int b = 0; b < NC; ++b) E[a][b] = pb[(PB_E + a * NC + b) * n + c];
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    Cn.Hv[i] = pb[(PB_HV + i) * n + c];
    Cn.He[i] = pb[(PB_HE + i) * n + c];
    Cn.Hs[i] = pb[(PB_HS + i) * n + c];
  }
  bool ok = chol_n<NC>(E, R);
  mldiv_spd<NC>(E, R, ok, F, y);
  ConsM Mf{Cn};
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    double sum = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) sum = sum + Mf(i, k) * y[k];
    K[i] = sum + pb[(PB_GAM + i) * n + c];
  }
}

// A finite dummy QP for lanes that only ride along (no QP this step / no queued cell).
__device__ __forceinline__ void hild_dummy(Cons &Cn, double E[NC][NC], double K[NCON]) {
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) E[a][b] = a == b ? 1.0 : 0.0;
#pragma unroll
  for (int i = 0; i < NP; ++i) Cn.Hv[i] = Cn.He[i] = Cn.Hs[i] = 0.0;
#pragma unroll
  for (int i = 0; i < NCON; ++i) K[i] = 0.0;
}

// DU = -E\(F + M'*lambda) (hildreth.m:46), then iterMPC.m:75-95 and the outputs.
__device__ __forceinline__ void hild_finish(const KState &s, const KIO &io, int64_t c, const Cons &Cn,
                                            const double Mtl[NC], int nexec) {
  const int64_t n = s.n;
  const double *pb = s.prob;
  asm volatile("" : "+v"(pb));  // operands re-read after the sweeps, not kept live across them
  MpcOut o;
  o.nexec = nexec;
  MpcSetup P;
  double rhs[NC], mE[NC][NC];
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    rhs[a] = pb[(PB_F + a) * n + c] + Mtl[a];
#pragma unroll
    for (int b = 0; b < NC; ++b) mE[a][b] = -pb[(PB_E + a * NC + b) * n + c];
  }
  lu_solve_n<NC>(mE, rhs, P.DU);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    P.e[i] = pb[(PB_ERR + i) * n + c];
    P.Cn.Hv[i] = Cn.Hv[i];
    P.Cn.He[i] = Cn.He[i];
    P.Cn.Hs[i] = Cn.Hs[i];
  }
#pragma unroll
  for (int i = 0; i < NCON; ++i) P.Cn.gam[i] = pb[(PB_GAM + i) * n + c];
  P.Ru = pb[PB_RU * n + c];
  double uk_1 = pb[PB_UK1 * n + c];
  mpc_finish(P.Cn, P.e, P.Ru, P.DU, uk_1, o);
  s.uk_1[c] = uk_1;
  if (s.J_fin) { s.J_fin[c] = o.J_fin; s.nviol[c] = o.nviol; }
  cost_out(io, c, o.J_fin, o.nviol, norm_du<NC>(P.DU));
  if (io.uk_out) io.uk_out[c] = o.uk;
  if (io.nexec) io.nexec[c] = o.nexec;
  if (io.mode & MODE_FUSED) {
    s.uk[c] = o.uk;
    if (io.u) io.u[c] = o.uk;
  }
}

__device__ __forceinline__ void hild_slow_cell(const KCfg &cf, const KState &s, const KIO &io, int64_t c);
// out of line: the exact-rule path keeps its registers out of the fast sweep's allocation
__device__ __noinline__ void hild_slow_wave(const KCfg &cf, const KState &s, const KIO &io, int64_t c) {
  hild_slow_cell(cf, s, io, c);
}

// hildreth.m + iterMPC.m:68-95, lane per cell: the fast solve (hild_fast).  Blocks of 256
// lanes (hild_lane_lds); k_hild, or the end of k_cell in the fused step.
__device__ __forceinline__ void hild_cell(const KCfg &cf, const KState &s, const KIO &io, int64_t c) {
  // every lane of the wave stays in the solve; cells without a QP this step ride
  // along on a finite dummy problem and store nothing
  const bool qp = s.hflag[c] != 0;
  const int64_t n = s.n;
  Cons Cn;
  double E[NC][NC], K[NCON], lam[NCON];
  if (!qp) {
    hild_dummy(Cn, E, K);
#pragma unroll
    for (int i = 0; i < NCON; ++i) lam[i] = 0.0;
  } else {
    hild_load(s, c, Cn, E, K);
#pragma unroll
    for (int i = 0; i < NCON; ++i) lam[i] = s.lam[(size_t)i * n + c];
  }
  extern __shared__ double2 hlds[];
  int nexec;
  const bool slow = hild_fast(Cn, E, lam, cf.max_hild, cf.hild_tol, K, !qp, hild_lane_lds(hlds), s.lam + c, n, nexec);
  if (MPCEKF_HILD_INLINE_SLOW) {
    // the rare wave with a lane outside the fast form's domain redoes that lane with the
    // exact rules here (warm start still in s.lam), the wave's other lanes riding along on
    // the dummy problem: no second kernel, whose launch cost ~4 us a step even when empty
    if (qp && slow) s.hflag[c] = 2;
    if (__any(slow)) hild_slow_wave(cf, s, io, c);
    if (!qp || slow) return;
  } else {
    if (__any(slow) && (threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63))
      atomicAdd(s.hslow, 1);  // one add per wave: k_hild_slow has work
    if (!qp) return;
    if (slow) {  // k_hild_slow finishes it (warm start still in s.lam)
      s.hflag[c] = 2;
      return;
    }
  }
  double Mtl[NC];
  hild_mtl(Cn, lam, Mtl);
#pragma unroll
  for (int i = 0; i < NCON; ++i) s.lam[(size_t)i * n + c] = lam[i];  // iterMPC.m:68
  hild_finish(s, io, c, Cn, Mtl, nexec);
}
__global__ void __launch_bounds__(256) k_hild(const KCfg cf, const KState s, const KIO io) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= s.n) return;
  hild_cell(cf, s, io, c);
}

// The exact-rule solve of the cells k_hild flagged (hflag 2): one wave per block over a
// grid-stride range of waves, gone at once when k_hild counted none.
__device__ __forceinline__ void hild_slow_cell(const KCfg &cf, const KState &s, const KIO &io, int64_t c);
__global__ void __launch_bounds__(64) k_hild_slow(const KCfg cf, const KState s, const KIO io) {
  if (__builtin_amdgcn_readfirstlane(*s.hslow) == 0) return;
  for (int64_t w = blockIdx.x; w * 64 < s.n; w += gridDim.x) hild_slow_cell(cf, s, io, w * 64 + threadIdx.x);
}
__device__ __forceinline__ void hild_slow_cell(const KCfg &cf, const KState &s, const KIO &io, int64_t c) {
  if (c >= s.n) return;
  const bool slow = s.hflag[c] == 2;
  if (!__any(slow)) return;
  const int64_t n = s.n;
  Cons Cn;
  double E[NC][NC], K[NCON], lam[NCON];
  if (!slow) {
    hild_dummy(Cn, E, K);
#pragma unroll
    for (int i = 0; i < NCON; ++i) lam[i] = 0.0;
  } else {
    hild_load(s, c, Cn, E, K);
#pragma unroll
    for (int i = 0; i < NCON; ++i) lam[i] = s.lam[(size_t)i * n + c];
  }
  extern __shared__ double2 hlds[];
  const int nexec = hild_slow(Cn, E, lam, cf.max_hild, cf.hild_tol, K, !slow, hild_lane_lds(hlds));
  if (!slow) return;
  s.hflag[c] = 1;
  double Mtl[NC];
  hild_mtl(Cn, lam, Mtl);
#pragma unroll
  for (int i = 0; i < NCON; ++i) s.lam[(size_t)i * n + c] = lam[i];
  hild_finish(s, io, c, Cn, Mtl, nexec);
}

// ---------------------------------------------------------------------------
// context-free batched kernels
// ---------------------------------------------------------------------------
__global__ void k_predmat(int64_t n, const double *a, const double *C, const double *D, double *Phi, double *G) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double av[6], Cb[7], P[NP][NA], H[NP];
#pragma unroll
  for (int k = 0; k < 6; ++k) { av[k] = a[c * 6 + k]; Cb[k] = C[c * 6 + k]; }
  Cb[6] = D[c];
  predmat_s(av, Cb, P, H);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
#pragma unroll
    for (int k = 0; k < NA; ++k) Phi[(c * NP + i) * NA + k] = P[i][k];
#pragma unroll
    for (int j = 0; j < NC; ++j) G[(c * NP + i) * NC + j] = j <= i ? H[i - j] : 0.0;
  }
}

__global__ void __launch_bounds__(64) k_constraints(const KCfg cf, int64_t n, const double *lin,
                                                    const double *uk_1, const double *soc_k1, double *Mo,
                                                    double *go) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  Lin L;
  lin_load(lin + c * 35, L);
  double dx[NA];
#pragma unroll
  for (int k = 0; k < 6; ++k) dx[k] = L.xhat[k];
  dx[6] = uk_1[c];
  double Phis[NP][NA], Hs[NP], Cb[7];
#pragma unroll
  for (int k = 0; k < 6; ++k) Cb[k] = L.Csoc[k];
  Cb[6] = L.Dsoc;
  predmat_s(L.a, Cb, Phis, Hs);
  Cons Cn;
  constraints_s(cf, L, dx, uk_1[c], soc_k1[c], Phis, Hs, Cn);
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    go[c * NCON + i] = Cn.gam[i];
#pragma unroll
    for (int j = 0; j < NC; ++j) Mo[(c * NCON + i) * NC + j] = mval(Cn, i, j);
  }
}

// hildreth.m for an arbitrary (E, F, M, gamma): M is data, not the pattern.
__global__ void __launch_bounds__(64) k_hildreth(int64_t n, const double *Ei, const double *Fi, const double *Mi,
                                                 const double *gi, double *lami, int maxIter, double tol,
                                                 double *DUo, int *nexec) {
  int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double E[NC][NC], F[NC], M[NCON][NC], gam[NCON], lam[NCON], DU[NC];
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    F[a] = Fi[c * NC + a];
#pragma unroll
    for (int b = 0; b < NC; ++b) E[a][b] = Ei[(c * NC + a) * NC + b];
  }
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    gam[i] = gi[c * NCON + i];
    lam[i] = lami[c * NCON + i];
#pragma unroll
    for (int j = 0; j < NC; ++j) M[i][j] = Mi[(c * NCON + i) * NC + j];
  }
  DenseM Mf{M};
  int it = hildreth_core(Mf, E, F, gam, lam, maxIter, tol, DU);
#pragma unroll
  for (int i = 0; i < NCON; ++i) lami[c * NCON + i] = lam[i];
#pragma unroll
  for (int a = 0; a < NC; ++a) DUo[c * NC + a] = DU[a];
  nexec[c] = it;
}

// hildreth.m for any Nc <= HANY_NC and nC <= HANY_NCON with a dense M (mpcekf_hildreth at
// sizes other than the fused Np = 5 / Nc = 2): orc_hildreth's defined evaluation with
// runtime sizes, lane per problem.  X = E\M' (Cholesky, else LU), H_ii and K live in a
// per-problem scratch slab; the dense path re-forms H(i,j) entry by entry.  A stage entry
// point, not the fused path: sized for correctness, not speed.
constexpr int HANY_NC = 10, HANY_NCON = 100;
__device__ inline bool chol_rt(int n, const double *E, double *R) {
  bool ok = true;
  for (int j = 0; j < n; ++j) {
    double s = E[j * n + j];
    for (int k = 0; k < j; ++k) s = s - R[k * n + j] * R[k * n + j];
    if (!(s > 0)) ok = false;
    R[j * n + j] = sqrt(s);
    for (int i = j + 1; i < n; ++i) {
      double t = E[j * n + i];
      for (int k = 0; k < j; ++k) t = t - R[k * n + j] * R[k * n + i];
      R[j * n + i] = t / R[j * n + j];
    }
  }
  return ok;
}
__device__ inline void lu_rt(int n, const double *Ain, const double *b, double *x) {
  double A[HANY_NC * HANY_NC], y[HANY_NC];
  for (int i = 0; i < n * n; ++i) A[i] = Ain[i];
  for (int i = 0; i < n; ++i) y[i] = b[i];
  for (int k = 0; k < n; ++k) {
    int p = k;
    for (int i = k + 1; i < n; ++i)
      if (fabs(A[i * n + k]) > fabs(A[p * n + k])) p = i;
    if (p != k) {
      for (int j = 0; j < n; ++j) { const double t = A[k * n + j]; A[k * n + j] = A[p * n + j]; A[p * n + j] = t; }
      const double t = y[k]; y[k] = y[p]; y[p] = t;
    }
    for (int i = k + 1; i < n; ++i) {
      const double l = A[i * n + k] / A[k * n + k];
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
// MATLAB E\b for symmetric E: Cholesky when every pivot is positive, else LU
__device__ inline void mldiv_rt(int n, const double *E, const double *R, bool ok, const double *b, double *x) {
  if (!ok) {
    lu_rt(n, E, b, x);
    return;
  }
  double y[HANY_NC];
  for (int i = 0; i < n; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t = t - R[k * n + i] * y[k];
    y[i] = t / R[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = y[i];
    for (int k = i + 1; k < n; ++k) t = t - R[i * n + k] * x[k];
    x[i] = t / R[i * n + i];
  }
}
// t_i = K_i + M(i,:)*v (orc hild_row_t): Nc <= 2 fma in ascending k; else the 8-lane
// form: a_0 = fma(M_i0, v_0, K_i), a_k = M_ik v_k (+0 past Nc), b_k = fma(M_i,k+8, v_k+8, a_k)
// while k + 8 < Nc, then the pairwise tree over the 8 slots
__device__ inline double row_t_rt(int Nc, const double *Mi, const double *v, double Ki) {
  if (Nc <= 2) {
    double t = Ki;
    for (int k = 0; k < Nc; ++k) t = __builtin_fma(Mi[k], v[k], t);
    return t;
  }
  double b[8];
  for (int k = 0; k < 8; ++k) {
    const double a = k == 0 ? __builtin_fma(Mi[0], v[0], Ki) : (k < Nc ? Mi[k] * v[k] : 0.0);
    b[k] = k + 8 < Nc ? __builtin_fma(Mi[k + 8], v[k + 8], a) : a;
  }
  for (int w = 1; w < 8; w *= 2)
    for (int k = 0; k < 8; k += 2 * w) b[k] = b[k] + b[k + w];
  return b[0];
}
__global__ void __launch_bounds__(64) k_hildreth_any(int64_t n, int Nc, int nC, const double *Ei, const double *Fi,
                                                     const double *Mi, const double *gi, double *lami, int maxIter,
                                                     double tol, double *DUo, int *nexec, double *scr) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const double *E = Ei + (size_t)c * Nc * Nc, *F = Fi + (size_t)c * Nc, *M = Mi + (size_t)c * nC * Nc,
               *gam = gi + (size_t)c * nC;
  double *lam = lami + (size_t)c * nC;
  double *X = scr + (size_t)c * (nC * Nc + 2 * nC), *Hd = X + nC * Nc, *K = Hd + nC;
  double R[HANY_NC * HANY_NC], y[HANY_NC], v[HANY_NC];
  const bool ok = chol_rt(Nc, E, R);
  for (int i = 0; i < nC; ++i) mldiv_rt(Nc, E, R, ok, M + i * Nc, X + i * Nc);  // X(:,i) = E\M(i,:)'
  mldiv_rt(Nc, E, R, ok, F, y);
  bool fin = true;
  for (int i = 0; i < nC; ++i) {
    double s = 0.0, h = 0.0;
    for (int k = 0; k < Nc; ++k) {
      s = s + M[i * Nc + k] * y[k];
      h = h + M[i * Nc + k] * X[i * Nc + k];
      fin = fin && isfinite(X[i * Nc + k]) && isfinite(M[i * Nc + k]);
    }
    K[i] = s + gam[i];
    Hd[i] = h;
  }
  auto xv = [&]() {
    for (int k = 0; k < Nc; ++k) {
      double a = 0.0;
      for (int j = 0; j < nC; ++j) a = __builtin_fma(X[j * Nc + k], lam[j], a);
      v[k] = a;
    }
  };
  int it;
  for (it = 1; it <= maxIter; ++it) {
    bool conv = true;
    if (fin) xv();
    for (int i = 0; i < nC; ++i) {
      const double hii = Hd[i];
      double nl, d;
      if (fin) {
        const double t = row_t_rt(Nc, M + i * Nc, v, K[i]);
        d = hild_step(t, hii, 1.0 / hii, lam[i], nl);
      } else {
        double p4[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = 0; j < nC; ++j) {
          double h = 0.0;
          for (int k = 0; k < Nc; ++k) h = h + M[i * Nc + k] * X[j * Nc + k];
          p4[j & 3] = p4[j & 3] + h * lam[j];
        }
        const double s = (p4[0] + p4[1]) + (p4[2] + p4[3]);
        const double w = -((K[i] + s) - hii * lam[i]) / hii;
        nl = w > 0 ? w : 0.0;
        d = nl - lam[i];
      }
      if (!(fabs(d) < tol)) conv = false;
      lam[i] = nl;
      if (fin) {
        if (isfinite(d)) {
          for (int k = 0; k < Nc; ++k) v[k] = __builtin_fma(X[i * Nc + k], d, v[k]);
        } else {
          xv();
        }
      }
    }
    if (conv) break;
  }
  if (it > maxIter) it = maxIter;
  double rhs[HANY_NC], mE[HANY_NC * HANY_NC], DU[HANY_NC];
  for (int k = 0; k < Nc; ++k) {
    double s = 0.0;
    for (int i = 0; i < nC; ++i) s = s + M[i * Nc + k] * lam[i];
    rhs[k] = F[k] + s;
  }
  for (int i = 0; i < Nc * Nc; ++i) mE[i] = -E[i];
  lu_rt(Nc, mE, rhs, DU);
  for (int k = 0; k < Nc; ++k) DUo[(size_t)c * Nc + k] = DU[k];
  nexec[c] = it;
}

// The fused solver (hild_fast + hild_slow, as k_hild + k_hild_slow) on constraintsMPC.m-structured
// problems given by their Toeplitz rows: M = [Cu; -Cu; I; -I; G_v; -G_e; G_soc].
template <bool SLOW>
__global__ void __launch_bounds__(256) k_hildreth_structured(int64_t n, const double *Ei, const double *Fi,
                                                             const double *Hvi, const double *Hei,
                                                             const double *Hsi, const double *gi, double *lami,
                                                             int maxIter, double tol, double *DUo, int *nexec) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool real = c < n;  // lanes past n ride along (hild_fast keeps the wave full)
  const int64_t cc = real ? c : 0;
  Cons Cn;
  double E[NC][NC], F[NC], K[NCON], lam[NCON];
  if (!real) {
    hild_dummy(Cn, E, K);
#pragma unroll
    for (int i = 0; i < NCON; ++i) lam[i] = 0.0;
#pragma unroll
    for (int a = 0; a < NC; ++a) F[a] = 0.0;
  } else {
#pragma unroll
    for (int a = 0; a < NC; ++a) {
      F[a] = Fi[cc * NC + a];
#pragma unroll
      for (int b = 0; b < NC; ++b) E[a][b] = Ei[(cc * NC + a) * NC + b];
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      Cn.Hv[i] = Hvi[cc * NP + i];
      Cn.He[i] = Hei[cc * NP + i];
      Cn.Hs[i] = Hsi[cc * NP + i];
    }
    double y[NC], R[NC][NC];
    bool ok = chol_n<NC>(E, R);
    mldiv_spd<NC>(E, R, ok, F, y);
    ConsM Mf{Cn};
#pragma unroll
    for (int i = 0; i < NCON; ++i) {
      double sum = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) sum = sum + Mf(i, k) * y[k];
      K[i] = sum + gi[cc * NCON + i];
      lam[i] = lami[cc * NCON + i];
    }
  }
  extern __shared__ double2 hlds[];
  int it;
  bool slow = false;
  if (SLOW) {
    slow = real && nexec[cc] < 0;
    if (!__any(slow)) return;
    if (!slow) {  // a finished problem rides along as a passenger
      hild_dummy(Cn, E, K);
#pragma unroll
      for (int i = 0; i < NCON; ++i) lam[i] = 0.0;
    }
    it = hild_slow(Cn, E, lam, maxIter, tol, K, !slow, hild_lane_lds(hlds));
    if (!slow) return;
  } else {
    if (hild_fast(Cn, E, lam, maxIter, tol, K, !real, hild_lane_lds(hlds), lami + cc * NCON, 1, it)) {
      if (real) nexec[cc] = -1;  // the second launch finishes it (warm start still in lambda)
      return;
    }
  }
  double Mtl[NC];
  hild_mtl(Cn, lam, Mtl);
  if (!real) return;
  double rhs[NC], mE[NC][NC], DU[NC];
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    rhs[a] = F[a] + Mtl[a];
#pragma unroll
    for (int b = 0; b < NC; ++b) mE[a][b] = -E[a][b];
  }
  lu_solve_n<NC>(mE, rhs, DU);
#pragma unroll
  for (int i = 0; i < NCON; ++i) lami[cc * NCON + i] = lam[i];
#pragma unroll
  for (int a = 0; a < NC; ++a) DUo[cc * NC + a] = DU[a];
  nexec[cc] = it;
}

// initKF.m:94-95 / OB_step.m:185: xhat = 0, SigmaX = SigmaX0(1:5,1:5), bigX = 0
__global__ void k_init_state(int64_t n, int NM, double *ekf, double *bigx, double s0, double s1, double s2, double s3,
                             double s4) {
  const double d[NX] = {s0, s1, s2, s3, s4};
  int64_t total = n * NM;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    double *rec = ekf + i * REC;
#pragma unroll
    for (int k = 0; k < NX; ++k) rec[k] = 0.0;
#pragma unroll
    for (int p = 0; p < NX; ++p)
#pragma unroll
      for (int q = p; q < NX; ++q) rec[NX + pk(p, q)] = p == q ? d[p] : 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) bigx[i * 6 + k] = 0.0;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int launch_init_state(int64_t n, int NM, double *ekf, double *bigx, const double *sx0, void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_init_state, dim3(2048), dim3(256), 0, (hipStream_t)stream, n, NM, ekf, bigx, sx0[0], sx0[1],
                     sx0[2], sx0[3], sx0[4]);
  return (int)hipGetLastError();
}
static int grid_for(int64_t n, int block) { return (int)((n + block - 1) / block); }

// Compute units of the current device (cached per device).
static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}
// Block size of a kernel whose blocks each take a CU's LDS (k_cell's ROM blob, k_hild's slots,
// k_bounds' model blob), lpc lanes per cell, launch bound maxb: the fewest 64-lane waves per
// block that still cover the batch in one round of blocks over the CUs.  A small batch then
// runs one wave per CU (configs[1]: 16 CUs) instead of four waves on each of n/256 CUs sharing
// the CU's LDS, L1 and address units; from 64 x #CUs x 4 lanes up it is maxb as before.
// MPCEKF_SPREAD=0: always maxb (A/B; results identical, every lane's arithmetic is its own).
static int spread_block(int64_t n, int lpc, int maxb) {
  const char *e = std::getenv("MPCEKF_SPREAD");  // read per launch: tests toggle it in-process
  if (e && std::atoi(e) == 0) return maxb;
  const int64_t lanes = n * lpc, cus = cu_count();
  int64_t b = (lanes + cus - 1) / cus;
  b = (b + 63) / 64 * 64;
  return (int)(b < 64 ? 64 : b > maxb ? maxb : b);
}

int cell_lds_bytes(const KRom &r) {
  return (int)((r.cell_len - (r.rom_global ? r.cell_tab : 0) + 1) * sizeof(double));
}
int bounds_lds_bytes(const KRom &r, int block) { return (bounds_c0_base(r) + block / 4 * 8) * (int)sizeof(double); }
int plant_lds_bytes(const KRom &r) {
  return (int)((r.plant_len - (r.rom_global ? r.plant_tab : 0) + 1) * sizeof(double));
}

bool cell_kernel_supported(int nzp) { return nzp == 26 || nzp == 32; }

int launch_plant(const KRom &r, const KState &s, const double *iapp, double *vout, int lazy_t, const double *tc_in,
                 void *stream) {
  if (s.n == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  const int lds = plant_lds_bytes(r);
  if (MPCEKF_PLANT_QUAD) {
    const int block = spread_block(s.n, 4, PLANT4_BLOCK);
    const dim3 g(grid_for(4 * s.n, block)), b(block);
    if (r.npoly) {
      if (r.rom_global) hipLaunchKernelGGL((k_plant4<true, true>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
      else hipLaunchKernelGGL((k_plant4<false, true>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
    } else {
      if (r.rom_global) hipLaunchKernelGGL((k_plant4<true, false>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
      else hipLaunchKernelGGL((k_plant4<false, false>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
    }
    return (int)hipGetLastError();
  }
  const dim3 g(grid_for(s.n, 256)), b(256);
  if (r.npoly) {
    if (r.rom_global) hipLaunchKernelGGL((k_plant<true, true>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
    else hipLaunchKernelGGL((k_plant<false, true>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
  } else {
    if (r.rom_global) hipLaunchKernelGGL((k_plant<true, false>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
    else hipLaunchKernelGGL((k_plant<false, false>), g, b, lds, st, r, s, iapp, vout, lazy_t, tc_in);
  }
  return (int)hipGetLastError();
}

int launch_flush(const KRom &r, const KCfg &c, const KState &s, int t, int new_ts, void *stream, int64_t c_lo,
                 int64_t c_hi) {
  if (c_hi < 0 || c_hi > s.n) c_hi = s.n;
  if (c_lo < 0) c_lo = 0;
  if (c_hi <= c_lo) return 0;
  static_assert((LAZY_H & (LAZY_H - 1)) == 0 && LAZY_H <= 64, "k_flush: ring slots live in lanes");
  // persistent waves striding over cells, as many as fit: 2 per SIMD with the pipelined
  // loads (210 VGPRs), 3 without (150)
  const int64_t wmax = MPCEKF_FLUSH_PF ? 2048 : 3072;
  const int64_t waves = c_hi - c_lo < wmax ? c_hi - c_lo : wmax;
  if (MPCEKF_FLUSH_COAL && r.NM <= 64)
    hipLaunchKernelGGL(k_flush_coal, dim3((int)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream, r, c, s, t,
                       new_ts, c_lo, c_hi);
  else
    hipLaunchKernelGGL(k_flush, dim3((int)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream, r, c, s, t, new_ts,
                       c_lo, c_hi);
  return (int)hipGetLastError();
}

int launch_bulk(const KRom &r, const KCfg &c, const KState &s, const double *iapp, int do_plant, int do_ekf,
                void *stream) {
  if (s.n == 0) return 0;
  int lds = (int)((r.NM * REC + r.NM * 6) * sizeof(double));
  int grid = (int)(s.n < 2048 ? s.n : 2048);
  hipLaunchKernelGGL(k_bulk, dim3(grid), dim3(256), lds, (hipStream_t)stream, r, c, s, iapp, do_plant, do_ekf);
  return (int)hipGetLastError();
}

template <int NZ, int PARTS, bool MB, bool GR, bool PL>
static void launch_cell_g(const KRom &r, const KCfg &c, const KState &s, const KIO &io, hipStream_t st) {
  static bool attr = false;
  const int block = spread_block(s.n, 1, 256);
  int lds = cell_lds_bytes(r);
  const int hl = block / 64 * (int)HILD_LDS_PER_WAVE;
  if (io.hild) lds = lds > hl ? lds : hl;  // the Hildreth slots
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_cell<NZ, PARTS, MB, GR, PL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_cell<NZ, PARTS, MB, GR, PL>), dim3(grid_for(s.n, block)), dim3(block), lds, st, r, c, s, io);
}

template <int NZ, int PARTS, bool MB>
static void launch_cell_t(const KRom &r, const KCfg &c, const KState &s, const KIO &io, hipStream_t st) {
  if (r.npoly) {  // ABI v3 tables: the k_cell instantiations with the polynomial lookup
    if (r.rom_global)
      launch_cell_g<NZ, PARTS, MB, true, true>(r, c, s, io, st);
    else
      launch_cell_g<NZ, PARTS, MB, false, true>(r, c, s, io, st);
    return;
  }
  if (r.rom_global)
    launch_cell_g<NZ, PARTS, MB, true, false>(r, c, s, io, st);
  else
    launch_cell_g<NZ, PARTS, MB, false, false>(r, c, s, io, st);
}

template <int NZ>
static int launch_cell_nz(const KRom &r, const KCfg &c, const KState &s, const KIO &io, hipStream_t st, int parts) {
  if (c.flags & KF_MB) {  // the model-blend EKF ('MB'): fused 5/2, wide (EKF + linearisation) and all stages
    switch (parts) {
      case P_ALL: launch_cell_t<NZ, P_ALL, true>(r, c, s, io, st); return 0;
      case P_EKF | P_LIN: launch_cell_t<NZ, P_EKF | P_LIN, true>(r, c, s, io, st); return 0;
      default: return -1;
    }
  }
  switch (parts) {
    case P_EKF: launch_cell_t<NZ, P_EKF, false>(r, c, s, io, st); return 0;
    case P_MPC: launch_cell_t<NZ, P_MPC, false>(r, c, s, io, st); return 0;
    case P_ALL: launch_cell_t<NZ, P_ALL, false>(r, c, s, io, st); return 0;
    case P_EKF | P_LIN: launch_cell_t<NZ, P_EKF | P_LIN, false>(r, c, s, io, st); return 0;
    default: return -1;
  }
}

int launch_cell(const KRom &r, const KCfg &c, const KState &s, const KIO &io, void *stream, int parts) {
  if (s.n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  int rc = -1;
  switch (r.nzp) {
    case 26: rc = launch_cell_nz<26>(r, c, s, io, st, parts); break;
    case 32: rc = launch_cell_nz<32>(r, c, s, io, st, parts); break;
    default: return -1;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

template <int NZ, int BLOCK, bool GR, bool PL>
static void launch_ekf4_g(const KRom &r, const KCfg &c, const KState &s, const KIO &io, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_ekf4<NZ, BLOCK, GR, PL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  // BLOCK is the launch bound; the 256 instantiation (512 registers, no spills) runs the
  // fewest waves per block that cover the batch in one round of CUs (spread_block)
  const int block = BLOCK == 256 ? spread_block(s.n, 4, 256) : BLOCK;
  hipLaunchKernelGGL((k_ekf4<NZ, BLOCK, GR, PL>), dim3(grid_for(s.n * 4, block)), dim3(block), cell_lds_bytes(r), st,
                     r, c, s, io);
}

template <int NZ, int BLOCK>
static void launch_ekf4_t(const KRom &r, const KCfg &c, const KState &s, const KIO &io, hipStream_t st) {
  if (r.npoly) {
    if (r.rom_global)
      launch_ekf4_g<NZ, BLOCK, true, true>(r, c, s, io, st);
    else
      launch_ekf4_g<NZ, BLOCK, false, true>(r, c, s, io, st);
    return;
  }
  if (r.rom_global)
    launch_ekf4_g<NZ, BLOCK, true, false>(r, c, s, io, st);
  else
    launch_ekf4_g<NZ, BLOCK, false, false>(r, c, s, io, st);
}

// block = 256 (the small-batch mapping: 512 registers, one wave per SIMD, spread over the
// CUs), 512 (128 cells, 256 VGPRs, 2 waves per SIMD) or 1024 (256 cells, 128 VGPRs, 4 waves
// per SIMD)
int launch_ekf4(const KRom &r, const KCfg &c, const KState &s, const KIO &io, void *stream, int block) {
  if (s.n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (r.nzp) {
    case 26:
      if (block == 1024) launch_ekf4_t<26, 1024>(r, c, s, io, st);
      else if (block == 512) launch_ekf4_t<26, 512>(r, c, s, io, st);
      else launch_ekf4_t<26, 256>(r, c, s, io, st);
      break;
    case 32:
      if (block == 1024) launch_ekf4_t<32, 1024>(r, c, s, io, st);
      else if (block == 512) launch_ekf4_t<32, 512>(r, c, s, io, st);
      else launch_ekf4_t<32, 256>(r, c, s, io, st);
      break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

template <int NZ, bool GR>
static void launch_bounds_g(const KRom &r, const KState &s, const double *bnd, double *zbk, hipStream_t st) {
  static bool attr = false;
  const int block = spread_block(s.n, 4, BOUNDS_BLOCK);
  int lds = bounds_lds_bytes(r, block);
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_bounds<NZ, GR>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_bounds<NZ, GR>), dim3(grid_for(4 * s.n, block)), dim3(block), lds, st, r, s, bnd, zbk);
}

template <int NZ>
static void launch_bounds_t(const KRom &r, const KState &s, const double *bnd, double *zbk, hipStream_t st) {
  if (r.rom_global)
    launch_bounds_g<NZ, true>(r, s, bnd, zbk, st);
  else
    launch_bounds_g<NZ, false>(r, s, bnd, zbk, st);
}

int launch_bounds(const KRom &r, const KState &s, const double *bnd, double *zbk, void *stream) {
  if (s.n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (r.nzp) {
    case 26: launch_bounds_t<26>(r, s, bnd, zbk, st); break;
    case 32: launch_bounds_t<32>(r, s, bnd, zbk, st); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

static int hild_lds_bytes(int block = 256) {  // 4 waves per 256-thread block; one block per CU (147 KiB of 160)
  static_assert(4 * HILD_LDS_PER_WAVE <= 160 * 1024, "Hildreth slots exceed the LDS");
  return block / 64 * HILD_LDS_PER_WAVE;
}

size_t hildreth_any_scratch(int64_t n, int Nc, int ncon) { return (size_t)n * (size_t)(ncon * Nc + 2 * ncon); }

int launch_cl_diag(const KCfg &c, int64_t n, const double *lin, const double *uk1, double *poles, double *sv,
                   void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL((k_cl_diag<NP, NC>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream, c, n, lin,
                     uk1, poles, sv);
  return (int)hipGetLastError();
}

int launch_hild(const KCfg &c, const KState &s, const KIO &io, void *stream) {
  if (s.n == 0) return 0;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_hild, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int block = spread_block(s.n, 1, 256);
  hipLaunchKernelGGL(k_hild, dim3(grid_for(s.n, block)), dim3(block), hild_lds_bytes(block), (hipStream_t)stream, c, s,
                     io);
  if (!MPCEKF_HILD_INLINE_SLOW) {
    const int gs = grid_for(s.n, 64) < 256 ? grid_for(s.n, 64) : 256;
    hipLaunchKernelGGL(k_hild_slow, dim3(gs), dim3(64), HILD_LDS_PER_WAVE, (hipStream_t)stream, c, s, io);
  }
  return (int)hipGetLastError();
}

int launch_predmat(int64_t n, int Np, int Nc, const double *a, const double *C, const double *D, double *Phi,
                   double *G, void *stream) {
  if (Np != NP || Nc != NC) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_predmat, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, a, C, D, Phi, G);
  return (int)hipGetLastError();
}

int launch_constraints(const KCfg &c, int64_t n, const double *lin, const double *uk_1, const double *soc_k1,
                       double *M, double *gam, void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_constraints, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, c, n, lin, uk_1,
                     soc_k1, M, gam);
  return (int)hipGetLastError();
}

int launch_hildreth(int64_t n, int Nc, int ncon, const double *E, const double *F, const double *M,
                    const double *gam, double *lam, int max_iter, double tol, double *DU, int *nexec,
                    void *stream, double *scratch) {
  if (n == 0) return 0;
  if (Nc != NC || ncon != NCON) {  // any other size: the runtime-sized form (scratch: hildreth_any_scratch)
    if (Nc < 1 || Nc > HANY_NC || ncon < 1 || ncon > HANY_NCON || !scratch) return -1;
    hipLaunchKernelGGL(k_hildreth_any, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, n, Nc, ncon, E, F, M,
                       gam, lam, max_iter, tol, DU, nexec, scratch);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(k_hildreth, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, n, E, F, M, gam, lam,
                     max_iter, tol, DU, nexec);
  return (int)hipGetLastError();
}

int launch_hildreth_structured(int64_t n, const double *E, const double *F, const double *Hv, const double *He,
                               const double *Hs, const double *gam, double *lam, int max_iter, double tol,
                               double *DU, int *nexec, void *stream) {
  if (n == 0) return 0;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_hildreth_structured<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void *)k_hildreth_structured<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(k_hildreth_structured<false>, dim3(grid_for(n, 256)), dim3(256), hild_lds_bytes(),
                     (hipStream_t)stream, n, E, F, Hv, He, Hs, gam, lam, max_iter, tol, DU, nexec);
  hipLaunchKernelGGL(k_hildreth_structured<true>, dim3(grid_for(n, 256)), dim3(256), hild_lds_bytes(),
                     (hipStream_t)stream, n, E, F, Hv, He, Hs, gam, lam, max_iter, tol, DU, nexec);
  return (int)hipGetLastError();
}

}  // namespace mk
