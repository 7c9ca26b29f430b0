// mpcekf_wide.hip -- the MPC stage at the wide horizons Np = 20 / Nc = 10
// (BASELINE.json configs[4]: "larger QP, more Hildreth iters").
//
// The fused step runs k_cell as iterEKF + EKFmatsHandler only (P_EKF | P_LIN) and
// hands the linearisation record to:
//   k_mpc_wide        lane per cell   iterMPC.m:17-66 (predMat.m x3, adaptive Ru,
//                                     unconstrained LS, constraintsMPC.m, violation
//                                     test) and, when hildreth.m must run, its setup
//                                     (hildreth.m:17-29): X = E\M', K, H_ii
//   k_hild_wide       16-lane group   hildreth.m:32-42 sweeps; lane k holds v_k and
//                     per cell        column k of X in registers, row values are
//                                     summed by a DPP butterfly (oracle hild_row_t)
//   k_hild_wide_slow  lane per cell   the exact rules (inf/NaN rows, non-finite X or
//                                     M, non-SPD E) from the warm start
//   k_mpc_wide_finish lane per cell   hildreth.m:46 DU = -E\(F + M'*lambda) and
//                                     iterMPC.m:75-95
// A cell's QP has nC = 4 Nc + 3 Np = 100 rows and rank-Nc H = M E^-1 M' (SURVEY.md
// §5): the rank form keeps v = X*lambda (Nc numbers) current, so a row costs O(Nc).
// Arithmetic is oracle/mpcekf_oracle.c's defined order, bit for bit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "mpcekf_kernels.hpp"
#include "mpcekf_mpc.hpp"

#pragma clang fp contract(off)

namespace mk {
namespace {

template <int NP, int NC>
struct W {
  static constexpr int NCON = 4 * NC + 3 * NP;
  // problem record, SoA [field][n]
  static constexpr int E = 0, F = E + NC * NC, HV = F + NC, HE = HV + NP, HS = HE + NP, GAM = HS + NP,
                       ERR = GAM + NCON, RU = ERR + NP, UK1 = RU + 1, N = UK1 + 1;
  static constexpr int HPW = NC - 1 + NP;          // one Toeplitz block, NC - 1 leading zeros
  static constexpr int CELL_LDS = 3 * NCON + 3 * HPW;  // doubles per cell in k_hild_wide
  static constexpr int GROUPS = 16;                // cells per 256-thread block
};

template <int NP, int NC>
__device__ __forceinline__ void load_cons(const double *pb, int64_t n, int64_t c, ConsT<NP, NC> &Cn,
                                          bool with_gam) {
  using T = W<NP, NC>;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    Cn.Hv[i] = pb[(T::HV + i) * n + c];
    Cn.He[i] = pb[(T::HE + i) * n + c];
    Cn.Hs[i] = pb[(T::HS + i) * n + c];
  }
  if (with_gam) {
#pragma unroll
    for (int i = 0; i < T::NCON; ++i) Cn.gam[i] = pb[(T::GAM + i) * n + c];
  }
}

template <int NP, int NC>
__device__ __forceinline__ void load_E(const double *pb, int64_t n, int64_t c, double E[NC][NC]) {
  using T = W<NP, NC>;
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) E[a][b] = pb[(T::E + a * NC + b) * n + c];
}

// ---------------------------------------------------------------------------
// k_mpc_wide: iterMPC.m:17-66 per cell, then hildreth.m:17-29 when it must run
// ---------------------------------------------------------------------------
template <int NP, int NC>
__global__ void __launch_bounds__(64) k_mpc_wide(const KCfg cf, const KState s, const KIO io, const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  if (c >= n) return;
  const bool fused = io.mode & MODE_FUSED;
  s.hflag[c] = 0;
  if (s.status[c] & ST_ERROR) {  // the fused step's iterEKF kernel already wrote NaN outputs
    if (!fused) {
      if (io.uk_out) io.uk_out[c] = __builtin_nan("");
      if (io.nexec) io.nexec[c] = 0;
    }
    return;
  }
  Lin L;
  lin_load(io.lin_in + c * 35, L);
  const double SOCk_1 = io.soc_k1_in[c];
  double uk_1 = s.uk_1[c];
  MpcSetupT<NP, NC> P;
  MpcOut o;
  const bool need = mpc_setup<NP, NC>(cf, L, uk_1, SOCk_1, P, o, w.smin);
  if (s.J_unc) s.J_unc[c] = o.J_unc;
  if (!need) {
    mpc_finish<NP, NC>(P.Cn, P.e, P.Ru, P.DU, uk_1, o);
    s.uk_1[c] = uk_1;
    if (s.J_fin) { s.J_fin[c] = o.J_fin; s.nviol[c] = o.nviol; }
    if (io.uk_out) io.uk_out[c] = o.uk;
    if (io.nexec) io.nexec[c] = 0;
    if (fused) {
      s.uk[c] = o.uk;
      if (io.u) io.u[c] = o.uk;
    }
    return;
  }
  double *pb = w.prob;
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    pb[(T::F + a) * n + c] = P.F[a];
#pragma unroll
    for (int b = 0; b < NC; ++b) pb[(T::E + a * NC + b) * n + c] = P.E[a][b];
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    pb[(T::HV + i) * n + c] = P.Cn.Hv[i];
    pb[(T::HE + i) * n + c] = P.Cn.He[i];
    pb[(T::HS + i) * n + c] = P.Cn.Hs[i];
    pb[(T::ERR + i) * n + c] = P.e[i];
  }
#pragma unroll
  for (int i = 0; i < NCON; ++i) pb[(T::GAM + i) * n + c] = P.Cn.gam[i];
  pb[T::RU * n + c] = P.Ru;
  pb[T::UK1 * n + c] = uk_1;
  // hildreth.m:28-29 as orc_hildreth: X(:,i) = E\M(i,:)' by Cholesky, H_ii = M(i,:)*X(:,i),
  // K = M*(E\F) + gamma.  A non-SPD E (LU fallback) or a non-finite X / M goes to the
  // exact lane-per-cell kernel, which builds all of this itself.
  double R[NC][NC];
  const bool ok = chol_n<NC>(P.E, R);
  bool fin = ok;
  if (ok) {
    double y[NC];
    chol_apply<NC>(R, P.F, y);
#pragma unroll
    for (int i = 0; i < NCON; ++i) {
      double b[NC], x[NC];
#pragma unroll
      for (int k = 0; k < NC; ++k) b[k] = mval(P.Cn, i, k);
      chol_apply<NC>(R, b, x);
      double h = 0.0, kk = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        h = h + b[k] * x[k];
        kk = kk + b[k] * y[k];
        fin = fin && isfinite(x[k]) && isfinite(b[k]);
        w.X[((size_t)i * n + c) * NC + k] = x[k];
      }
      w.hii[(size_t)i * n + c] = h;
      w.K[(size_t)i * n + c] = kk + P.Cn.gam[i];
    }
  }
  s.hflag[c] = fin ? 1 : 2;
}

// ---------------------------------------------------------------------------
// k_hild_wide: hildreth.m:32-42 with a 16-lane group per cell
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// Sum over the 16 lanes of a DPP row as the pairwise tree of hild_row_t: each level
// adds the partner's partial sum (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror); both partners add the same two values, so every lane ends with the
// same bits.
__device__ __forceinline__ double tree16(double a) {
  a = a + dpp64<0xB1>(a);
  a = a + dpp64<0x4E>(a);
  a = a + dpp64<0x141>(a);
  a = a + dpp64<0x140>(a);
  return a;
}

// M(i, k) of the constraintsMPC.m pattern for lane k (i compile-time); the Toeplitz
// rows read the cell's padded impulse responses hp (exact zeros in front).
template <int NP, int NC>
__device__ __forceinline__ double mrow(int i, int k, const double *hp) {
  using T = W<NP, NC>;
  if (i < NC) return k <= i ? 1.0 : 0.0;                     // Cu
  if (i < 2 * NC) return -((k <= i - NC) ? 1.0 : 0.0);       // -Cu
  if (i < 3 * NC) return (i - 2 * NC) == k ? 1.0 : 0.0;      // I
  if (i < 4 * NC) return -((i - 3 * NC) == k ? 1.0 : 0.0);   // -I
  const int b = (i - 4 * NC) / NP, r = (i - 4 * NC) % NP;
  const int kk = k < NC ? k : NC - 1;
  const double h = hp[b * T::HPW + (NC - 1) + r - kk];
  return b == 1 ? -h : h;                                    // G_v, -G_e, G_soc
}

template <int NP, int NC>
__global__ void __launch_bounds__(256) k_hild_wide(const KCfg cf, const KState s, const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  extern __shared__ double lds[];
  const int g = threadIdx.x >> 4, k = threadIdx.x & 15;
  const int64_t n = s.n, c = (int64_t)blockIdx.x * T::GROUPS + g;
  double *lam = lds + g * T::CELL_LDS, *Kl = lam + NCON, *hl = Kl + NCON, *hp = hl + NCON;
  const bool act = c < n && s.hflag[c] == 1;
  if (act) {
    for (int i = k; i < NCON; i += 16) {
      lam[i] = s.lam[(size_t)i * n + c];
      Kl[i] = w.K[(size_t)i * n + c];
      hl[i] = w.hii[(size_t)i * n + c];
    }
    for (int j = k; j < 3 * T::HPW; j += 16) {
      const int b = j / T::HPW, q = j % T::HPW;
      hp[j] = q < NC - 1 ? 0.0 : w.prob[(T::HV + b * NP + q - (NC - 1)) * n + c];
    }
  }
  __syncthreads();
  if (!act) return;
  const int kx = k < NC ? k : 0;
  double X[NCON];
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    const double x = w.X[((size_t)i * n + c) * NC + kx];
    X[i] = k < NC ? x : 0.0;
  }
  const double tol = cf.hild_tol;
  const int maxIter = cf.max_hild;
  int it;
  bool slow = false;
  for (it = 1; it <= maxIter; ++it) {
    double v = 0.0;  // v = X*lambda (orc hild_v: fma from +0 in ascending j)
#pragma unroll
    for (int j = 0; j < NCON; ++j) v = __builtin_fma(X[j], lam[j], v);
    bool conv = true;
#pragma unroll
    for (int i = 0; i < NCON; ++i) {
      const double m = mrow<NP, NC>(i, k, hp);
      const double a = k == 0 ? __builtin_fma(m, v, Kl[i]) : (k < NC ? m * v : 0.0);
      const double t = tree16(a);
      const double hii = hl[i], li = lam[i];
      const double wv = __builtin_fma(hii, li, -t) / hii;
      const double nl = wv > 0 ? wv : 0.0;
      const double d = nl - li;
      conv = conv && fabs(d) < tol;
      slow = slow || !isfinite(d);
      lam[i] = nl;
      v = __builtin_fma(X[i], d, v);
    }
    if (slow || conv) break;
  }
  // A non-finite step (a zero-diagonal row going to or from +inf) switches the reference
  // evaluation to recomputing v from lambda: k_hild_wide_slow redoes this cell from its
  // warm start, which is still in s.lam (every sweep before was bit-identical).
  if (slow) {
    if (k == 0) s.hflag[c] = 2;
    return;
  }
  if (it > maxIter) it = maxIter;
  for (int i = k; i < NCON; i += 16) s.lam[(size_t)i * n + c] = lam[i];
  if (k == 0) w.it[c] = it;
}

// ---------------------------------------------------------------------------
// k_hild_wide_slow: orc_hildreth with every rule, lane per cell (hflag == 2)
// ---------------------------------------------------------------------------
template <int NP, int NC>
__device__ __forceinline__ double row_t(const ConsT<NP, NC> &Cn, int i, const double v[NC], double Ki) {
  if (NC <= 2) {
    double t = Ki;
#pragma unroll
    for (int k = 0; k < NC; ++k) t = __builtin_fma(mval(Cn, i, k), v[k], t);
    return t;
  }
  double a[16];
  a[0] = __builtin_fma(mval(Cn, i, 0), v[0], Ki);
#pragma unroll
  for (int k = 1; k < 16; ++k) a[k] = k < NC ? mval(Cn, i, k) * v[k] : 0.0;
#pragma unroll
  for (int wd = 1; wd < 16; wd *= 2)
#pragma unroll
    for (int k = 0; k < 16; k += 2 * wd) a[k] = a[k] + a[k + wd];
  return a[0];
}

template <int NP, int NC>
__device__ __forceinline__ void hild_v_g(const double *X, int64_t n, int64_t c, const double *lam, double v[NC]) {
  constexpr int NCON = W<NP, NC>::NCON;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    double a = 0.0;
#pragma unroll 1
    for (int j = 0; j < NCON; ++j) a = __builtin_fma(X[((size_t)j * n + c) * NC + k], lam[(size_t)j * n + c], a);
    v[k] = a;
  }
}

template <int NP, int NC>
__global__ void __launch_bounds__(64) k_hild_wide_slow(const KCfg cf, const KState s, const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  if (c >= n || s.hflag[c] != 2) return;
  ConsT<NP, NC> Cn;
  load_cons<NP, NC>(w.prob, n, c, Cn, true);
  double E[NC][NC], F[NC], R[NC][NC], y[NC];
  load_E<NP, NC>(w.prob, n, c, E);
#pragma unroll
  for (int a = 0; a < NC; ++a) F[a] = w.prob[(T::F + a) * n + c];
  const bool ok = chol_n<NC>(E, R);
  mldiv_spd<NC>(E, R, ok, F, y);
  bool fin = true;
#pragma unroll 1
  for (int i = 0; i < NCON; ++i) {
    double b[NC], x[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) b[k] = mval(Cn, i, k);
    mldiv_spd<NC>(E, R, ok, b, x);
    double h = 0.0, kk = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      h = h + b[k] * x[k];
      kk = kk + b[k] * y[k];
      fin = fin && isfinite(x[k]) && isfinite(b[k]);
      w.X[((size_t)i * n + c) * NC + k] = x[k];
    }
    w.hii[(size_t)i * n + c] = h;
    w.K[(size_t)i * n + c] = kk + Cn.gam[i];
  }
  double *lam = s.lam;
  const double tol = cf.hild_tol;
  const int maxIter = cf.max_hild;
  int it;
  for (it = 1; it <= maxIter; ++it) {
    bool conv = true;
    double v[NC];
    if (fin) hild_v_g<NP, NC>(w.X, n, c, lam, v);
#pragma unroll 1
    for (int i = 0; i < NCON; ++i) {
      const double hii = w.hii[(size_t)i * n + c], Ki = w.K[(size_t)i * n + c];
      const double li = lam[(size_t)i * n + c];
      double wv;
      if (fin) {
        wv = __builtin_fma(hii, li, -row_t<NP, NC>(Cn, i, v, Ki)) / hii;
      } else {  // dense H(i,:)*lambda, 4 interleaved partial sums (orc_hildreth)
        double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
        for (int j = 0; j < NCON; ++j) {
          double h = 0.0;
#pragma unroll
          for (int k = 0; k < NC; ++k) h = h + mval(Cn, i, k) * w.X[((size_t)j * n + c) * NC + k];
          p[j & 3] = p[j & 3] + h * lam[(size_t)j * n + c];
        }
        const double sm = (p[0] + p[1]) + (p[2] + p[3]);
        wv = -((Ki + sm) - hii * li) / hii;
      }
      const double nl = wv > 0 ? wv : 0.0;
      const double d = nl - li;
      if (!(fabs(d) < tol)) conv = false;
      lam[(size_t)i * n + c] = nl;
      if (fin) {
        if (isfinite(d)) {
#pragma unroll
          for (int k = 0; k < NC; ++k) v[k] = __builtin_fma(w.X[((size_t)i * n + c) * NC + k], d, v[k]);
        } else {
          hild_v_g<NP, NC>(w.X, n, c, lam, v);
        }
      }
    }
    if (conv) break;
  }
  if (it > maxIter) it = maxIter;
  w.it[c] = it;
}

// ---------------------------------------------------------------------------
// k_mpc_wide_finish: hildreth.m:46 and iterMPC.m:75-95 for the cells that ran it
// ---------------------------------------------------------------------------
template <int NP, int NC>
__global__ void __launch_bounds__(64) k_mpc_wide_finish(const KCfg cf, const KState s, const KIO io,
                                                        const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  if (c >= n || s.hflag[c] == 0) return;
  const double *pb = w.prob;
  ConsT<NP, NC> Cn;
  load_cons<NP, NC>(pb, n, c, Cn, false);
  double Mtl[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) Mtl[k] = 0.0;
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    const double li = s.lam[(size_t)i * n + c];
#pragma unroll
    for (int k = 0; k < NC; ++k) Mtl[k] = Mtl[k] + mval(Cn, i, k) * li;
  }
  double E[NC][NC], mE[NC][NC], rhs[NC], DU[NC];
  load_E<NP, NC>(pb, n, c, E);
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    rhs[a] = pb[(T::F + a) * n + c] + Mtl[a];
#pragma unroll
    for (int b = 0; b < NC; ++b) mE[a][b] = -E[a][b];
  }
  lu_solve_n<NC>(mE, rhs, DU);
  double uk_1 = pb[T::UK1 * n + c];
  const double uk = DU[0] + uk_1;
  uk_1 = uk;
  int nviol = 0;
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + mval(Cn, i, j) * DU[j];
    if (acc - pb[(T::GAM + i) * n + c] > 1e-9) nviol++;
  }
  double e[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) e[i] = pb[(T::ERR + i) * n + c];
  const int it = w.it[c];
  s.uk_1[c] = uk_1;
  if (s.J_fin) {
    s.J_fin[c] = mpc_cost<NP, NC>(Cn.Hs, e, pb[T::RU * n + c], DU);
    s.nviol[c] = nviol;
  }
  if (io.uk_out) io.uk_out[c] = uk;
  if (io.nexec) io.nexec[c] = it;
  if (io.mode & MODE_FUSED) {
    s.uk[c] = uk;
    if (io.u) io.u[c] = uk;
  }
}

// GsocT*Gsoc and its sigma_min, as mpc_setup forms them for Csoc = [0 0 0 0 0 rr],
// Dsoc = 0 (EKFmatsHandler.m:43-45): the cache mpc_setup compares bitwise.
template <int NP, int NC>
__global__ void k_wide_smin(double rr, double a0, double a1, double a2, double a3, double a4, double *out) {
  const double a[6] = {a0, a1, a2, a3, a4, 1.0};
  const double Cb[7] = {0.0, 0.0, 0.0, 0.0, 0.0, rr, 0.0};
  double Phis[NP][NA], Hs[NP], GtG[NC][NC];
  predmat_s<NP>(a, Cb, Phis, Hs);
#pragma unroll
  for (int p = 0; p < NC; ++p)
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < NP; ++i) acc = acc + (p <= i ? Hs[i - p] : 0.0) * (q <= i ? Hs[i - q] : 0.0);
      GtG[p][q] = acc;
      out[p * NC + q] = acc;
    }
  out[NC * NC] = sigma_min_n<NC>(GtG);
}

// context-free predMat.m / constraintsMPC.m
template <int NP, int NC>
__global__ void k_predmat_wide(int64_t n, const double *a, const double *C, const double *D, double *Phi, double *G) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double av[6], Cb[7], P[NP][NA], H[NP];
#pragma unroll
  for (int k = 0; k < 6; ++k) { av[k] = a[c * 6 + k]; Cb[k] = C[c * 6 + k]; }
  Cb[6] = D[c];
  predmat_s<NP>(av, Cb, P, H);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
#pragma unroll
    for (int k = 0; k < NA; ++k) Phi[(c * NP + i) * NA + k] = P[i][k];
#pragma unroll
    for (int j = 0; j < NC; ++j) G[(c * NP + i) * NC + j] = j <= i ? H[i - j] : 0.0;
  }
}

template <int NP, int NC>
__global__ void __launch_bounds__(64) k_constraints_wide(const KCfg cf, int64_t n, const double *lin,
                                                         const double *uk_1, const double *soc_k1, double *Mo,
                                                         double *go) {
  constexpr int NCON = W<NP, NC>::NCON;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
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
  predmat_s<NP>(L.a, Cb, Phis, Hs);
  ConsT<NP, NC> Cn;
  constraints_s<NP, NC>(cf, L, dx, uk_1[c], soc_k1[c], Phis, Hs, Cn);
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    go[c * NCON + i] = Cn.gam[i];
#pragma unroll
    for (int j = 0; j < NC; ++j) Mo[(c * NCON + i) * NC + j] = mval(Cn, i, j);
  }
}

int grid(int64_t n, int block) { return (int)((n + block - 1) / block); }

template <int NP, int NC>
int hild_lds_bytes_w() {
  return W<NP, NC>::GROUPS * W<NP, NC>::CELL_LDS * (int)sizeof(double);
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers: one instantiation, Np = 20 / Nc = 10
// ---------------------------------------------------------------------------
#define WIDE_NP 20
#define WIDE_NC 10

bool wide_supported(int Np, int Nc) { return Np == WIDE_NP && Nc == WIDE_NC; }
int wide_prob_doubles(int Np, int Nc) { return wide_supported(Np, Nc) ? W<WIDE_NP, WIDE_NC>::N : 0; }

int launch_wide_smin(const KWide &w, double rr, const double *a, void *stream) {
  if (!wide_supported(w.Np, w.Nc)) return -1;
  hipLaunchKernelGGL((k_wide_smin<WIDE_NP, WIDE_NC>), dim3(1), dim3(1), 0, (hipStream_t)stream, rr, a[0], a[1], a[2],
                     a[3], a[4], w.smin);
  return (int)hipGetLastError();
}

int launch_mpc_wide(const KCfg &c, const KState &s, const KIO &io, const KWide &w, void *stream) {
  if (!wide_supported(w.Np, w.Nc)) return -1;
  if (s.n == 0) return 0;
  hipLaunchKernelGGL((k_mpc_wide<WIDE_NP, WIDE_NC>), dim3(grid(s.n, 64)), dim3(64), 0, (hipStream_t)stream, c, s, io,
                     w);
  return (int)hipGetLastError();
}

int launch_hild_wide(const KCfg &c, const KState &s, const KIO &io, const KWide &w, void *stream) {
  if (!wide_supported(w.Np, w.Nc)) return -1;
  if (s.n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int lds = hild_lds_bytes_w<WIDE_NP, WIDE_NC>();
  hipLaunchKernelGGL((k_hild_wide<WIDE_NP, WIDE_NC>), dim3(grid(s.n, W<WIDE_NP, WIDE_NC>::GROUPS)), dim3(256), lds,
                     st, c, s, w);
  hipLaunchKernelGGL((k_hild_wide_slow<WIDE_NP, WIDE_NC>), dim3(grid(s.n, 64)), dim3(64), 0, st, c, s, w);
  hipLaunchKernelGGL((k_mpc_wide_finish<WIDE_NP, WIDE_NC>), dim3(grid(s.n, 64)), dim3(64), 0, st, c, s, io, w);
  return (int)hipGetLastError();
}

int launch_predmat_wide(int64_t n, int Np, int Nc, const double *a, const double *C, const double *D, double *Phi,
                        double *G, void *stream) {
  if (!wide_supported(Np, Nc)) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL((k_predmat_wide<WIDE_NP, WIDE_NC>), dim3(grid(n, 256)), dim3(256), 0, (hipStream_t)stream, n, a,
                     C, D, Phi, G);
  return (int)hipGetLastError();
}

int launch_constraints_wide(const KCfg &c, int Np, int Nc, int64_t n, const double *lin, const double *uk_1,
                            const double *soc_k1, double *M, double *gam, void *stream) {
  if (!wide_supported(Np, Nc)) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL((k_constraints_wide<WIDE_NP, WIDE_NC>), dim3(grid(n, 64)), dim3(64), 0, (hipStream_t)stream, c,
                     n, lin, uk_1, soc_k1, M, gam);
  return (int)hipGetLastError();
}

}  // namespace mk
