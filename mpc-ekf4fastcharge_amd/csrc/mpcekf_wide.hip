// mpcekf_wide.hip -- the MPC stage at the wide horizons Np = 20 / Nc = 10
// (BASELINE.json configs[4]: "larger QP, more Hildreth iters").
//
// The fused step runs k_cell as iterEKF + EKFmatsHandler only (P_EKF | P_LIN) and
// hands the linearisation record to:
//   k_mpc_wide        lane per cell   iterMPC.m:17-66: predMat.m x3, adaptive Ru, the
//                                     unconstrained LS solve, constraintsMPC.m and the
//                                     violation test, streamed row by row (no M or
//                                     gamma arrays live); finishes cells that need no QP
//   k_hild_prep       lane per cell   hildreth.m:17-29: R = chol(E) (handed over), K =
//                                     M*(E\F) + gamma (MPCEKF_WIDE_XPRO=0: also X(:,i) =
//                                     E\M(i,:)' for the 80 distinct rows and H_ii)
//   k_hild_wide       8-lane group    X and H_ii from R in its prologue (XPRO), then the
//                     per cell        hildreth.m:32-42 sweeps: lane k holds v_k (and v_k+8)
//                                     and column k of X in registers; row values are summed
//                                     by a DPP butterfly (oracle hild_row_t)
//   k_hild_wide_slow  lane per cell   the exact rules (inf/NaN rows, non-finite X or M,
//                                     non-SPD E, divisions outside the fast form's
//                                     domain) from the warm start
//   k_mpc_wide_finish lane per cell   hildreth.m:46 DU = -E\(F + M'*lambda) and
//                                     iterMPC.m:75-95
// A cell's QP has nC = 4 Nc + 3 Np = 100 rows and rank-Nc H = M E^-1 M' (SURVEY.md
// §5): the rank form keeps v = X*lambda (Nc numbers) current, so a row costs O(Nc).
// Arithmetic is oracle/mpcekf_oracle.c's defined order, bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>

#ifndef MPCEKF_WIDE_PF
#define MPCEKF_WIDE_PF 2     // k_hild_wide: rows of LDS operand prefetch
#endif
#ifndef PREP_UNROLL
#define PREP_UNROLL 1  // k_hild_prep's row loops (rows in flight per wave)
#endif
#ifndef MPCEKF_WIDE_SORT
#define MPCEKF_WIDE_SORT 1
#endif
// 1: k_hild_wide forms X(:,i) = E\M(i,:)' and H_ii itself from chol(E) (k_hild_prep hands
// over R, 55 doubles per cell, instead of writing X, 800, to HBM for k_hild_wide to read
// back); 0: k_hild_prep writes X and H_ii
#ifndef MPCEKF_WIDE_XPRO
#define MPCEKF_WIDE_XPRO 1
#endif
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
  // X is kept for the distinct rows only: [Cu (NC); I (NC); G_v, -G_e, G_soc (3 NP)];
  // the -Cu / -I rows use -X (E\(-b) = -(E\b) up to the sign of zero entries, which
  // never reaches a result: every sum they enter starts from +0).
  static constexpr int NX_ROWS = 2 * NC + 3 * NP;
  static constexpr int HPW = NC - 1 + NP;             // one Toeplitz block, NC - 1 leading zeros
  // k_hild_wide: 8 lanes per cell (lane k holds columns k and k + 8 of X), 16 cells per
  // 128-thread block.  Doubles per cell, even: each group's (H_ii, 1/H_ii) pairs are read
  // with ds_read_b128, which on a 16-byte-misaligned address costs ~15x an aligned read
  // (tools/micro/lds_micro.hip); the stride is 4 (mod 32) doubles, so the 8 groups of a
  // wave reading one offset of their own regions hit 8 disjoint bank pairs (b64) / quads (b128)
  static constexpr int CELL_LDS = (4 * NCON + 3 * HPW + 1 - 4 + 31) / 32 * 32 + 4;
  static constexpr int ZERO_LDS = (NCON + 1) & ~1;    // the zero row ahead of the groups
  static constexpr int LANES = 8;                     // lanes per cell
  static constexpr int BLOCK = 128;
  static constexpr int GROUPS = BLOCK / LANES;        // cells per block
  static constexpr int JUNK = 64 + NCON;              // per-wave sink of the lanes k != 0's lambda stores
  static constexpr int WAVES = BLOCK / 64;

};

// k_hild_sort's bins over last step's sweep count (0 .. maxIter)
constexpr int SWEEP_BINS = 64;
__device__ __forceinline__ int sweep_bin(int it, int maxIter) {
  if (!MPCEKF_WIDE_SORT) return 0;
  const int m = maxIter > 0 ? maxIter : 1;
  const int t = it < 0 ? 0 : it > m ? m : it;
  return (int)(((long long)t * SWEEP_BINS) / (m + 1));
}

// distinct-row slot of constraint row i, and whether row i is the negated copy
template <int NP, int NC>
__device__ __forceinline__ constexpr int xslot(int i) {
  return i < NC ? i : i < 2 * NC ? i - NC : i < 3 * NC ? i - NC : i < 4 * NC ? i - 2 * NC : i - 2 * NC;
}
template <int NC>
__device__ __forceinline__ constexpr bool xneg(int i) {
  return (i >= NC && i < 2 * NC) || (i >= 3 * NC && i < 4 * NC);
}

// One step k of predmat_s's recurrence: H(k) and row k of Phi.
__device__ __forceinline__ void pred_step(const double a[6], const double Cb[7], double S[6], double P[6], double &H,
                                          double row[7]) {
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) acc = acc + Cb[j] * S[j];
  acc = acc + Cb[6] * 1.0;
  H = acc;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    S[j] = a[j] * S[j] + 1.0;
    P[j] = a[j] * P[j];
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) row[j] = 0.0 + Cb[j] * P[j];
  double acc2 = 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) acc2 = acc2 + Cb[j] * S[j];
  row[6] = acc2 + Cb[6] * 1.0;
}
__device__ __forceinline__ double rowdot(const double row[7], const double dx[7]) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < NA; ++k) acc = acc + row[k] * dx[k];
  return acc;
}

// M(i, j) of the constant rows [Cu; -Cu; I; -I] (constraintsMPC.m:23-42), mval's literals
template <int NC>
__device__ __forceinline__ double mconst(int i, int j) {
  if (i < NC) return j <= i ? 1.0 : 0.0;
  if (i < 2 * NC) return -((j <= i - NC) ? 1.0 : 0.0);
  if (i < 3 * NC) return (i - 2 * NC) == j ? 1.0 : 0.0;
  return -((i - 3 * NC) == j ? 1.0 : 0.0);
}

template <int NP, int NC>
__device__ __forceinline__ void load_E(const double *pb, int64_t n, int64_t c, double E[NC][NC]) {
  using T = W<NP, NC>;
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) E[a][b] = pb[(T::E + a * NC + b) * n + c];
}

// sigma_min of GsocT*Gsoc out of line, from the copy k_mpc_wide left in the record's E
// slots: GsocT*Gsoc is a batch constant (the cached value hits), so the Jacobi runs only
// for foreign linearisations and must not add to k_mpc_wide's registers.
template <int NC>
__device__ __noinline__ double sigma_min_cold(const double *g, int64_t n) {
  double G[NC][NC];
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) G[a][b] = g[(size_t)(a * NC + b) * n];
  return sigma_min_n<NC>(G);
}

// ---------------------------------------------------------------------------
// k_mpc_wide: iterMPC.m:17-66 per cell (mpc_setup's arithmetic, streamed)
// ---------------------------------------------------------------------------
template <int NP, int NC>
__global__ void __launch_bounds__(64) k_mpc_wide(const KCfg cf, const KState s, const KIO io, const KWide w) {
  using T = W<NP, NC>;
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
  double *pb = w.prob;
  Lin L;
  lin_load(io.lin_in + c * 35, L);
  const double SOCk_1 = io.soc_k1_in[c];
  const double uk_1 = s.uk_1[c];
  double dx[NA];
#pragma unroll
  for (int k = 0; k < 6; ++k) dx[k] = L.xhat[k];
  dx[6] = uk_1;
  // predMat(Csoc): Hs, e = Ref - Phi_soc*dx (iterMPC.m:20-35); the SOC constraint rows'
  // gamma (constraintsMPC.m:89-101) from the same Phi_soc*dx
  double Hs[NP], e[NP], gs[NP];
  {
    double S[6], P[6], Cb[7], row[7];
#pragma unroll
    for (int j = 0; j < 6; ++j) { S[j] = 0.0; P[j] = 1.0; Cb[j] = L.Csoc[j]; }
    Cb[6] = L.Dsoc;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      pred_step(L.a, Cb, S, P, Hs[k], row);
      const double acc = rowdot(row, dx);
      e[k] = cf.ref * 1.0 - acc;
      gs[k] = cf.zmax * 1.0 - (acc + SOCk_1 * 1.0);
    }
  }
  double F[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) acc = acc + (-2 * (j <= i ? Hs[i - j] : 0.0)) * e[i];
    F[j] = acc;
  }
  // E = 2(G'G + Ru I), Ru = ||F|| / (2 du_max sqrt(Nc)) - sigma_min(G'G) (iterMPC.m:38-47).
  // G'G is formed twice (for the sigma_min cache test, then for E) rather than kept live.
  auto gtg = [&](int a, int b) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) acc = acc + (a <= i ? Hs[i - a] : 0.0) * (b <= i ? Hs[i - b] : 0.0);
    return acc;
  };
  bool hit = true;
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) {
      const double gab = gtg(a, b);
      hit = hit && __double_as_longlong(gab) == __double_as_longlong(w.smin[a * NC + b]);
      pb[(T::E + a * NC + b) * n + c] = gab;
    }
  const double smin = hit ? w.smin[NC * NC] : sigma_min_cold<NC>(pb + T::E * n + c, n);
  double nF = 0.0;
#pragma unroll
  for (int j = 0; j < NC; ++j) nF = nF + F[j] * F[j];
  nF = sqrt(nF);
  const double Ru = (nF / (2 * cf.du_max * sqrt((double)NC))) - smin;
  double mE[NC][NC], DU[NC];
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    pb[(T::F + a) * n + c] = F[a];
#pragma unroll
    for (int b = 0; b < NC; ++b) {
      const double eab = 2 * (gtg(a, b) + Ru * (a == b ? 1.0 : 0.0));
      pb[(T::E + a * NC + b) * n + c] = eab;
      mE[a][b] = -eab;
    }
  }
  lu_solve_n<NC>(mE, F, DU);  // DU = -E\F (iterMPC.m:48)
  const double J_unc = mpc_cost<NP, NC>(Hs, e, Ru, DU);
  if (s.J_unc) s.J_unc[c] = J_unc;
  if (io.junc_out) io.junc_out[c] = J_unc;
  // constraintsMPC.m rows: gamma to the record, M*DU - gamma tested as each row is formed
  int nv = 0, nviol = 0;
  // the row loops stay rolled (instruction fetch, see k_hild_prep); the G_v / -G_e rows'
  // M(k, :) is a shift register of the H column with mrow_vec's values
#pragma unroll 1
  for (int i = 0; i < 4 * NC; ++i) {
    const double g = i < NC ? (cf.u_max - uk_1) * 1.0 : i < 2 * NC ? -(cf.u_min - uk_1) * 1.0
                   : i < 3 * NC ? cf.du_max * 1.0 : -cf.du_min * 1.0;
    pb[(T::GAM + i) * n + c] = g;
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + mconst<NC>(i, j) * DU[j];
    if (acc - g > 0) nv++;
    if (acc - g > 1e-9) nviol++;
  }
  {  // G_v rows: predMat(Cv, Dv), gamma = v_max - (Phi_v*dx + bv)
    double S[6], P[6], Cb[7], row[7], b[NC];
#pragma unroll
    for (int j = 0; j < 6; ++j) { S[j] = 0.0; P[j] = 1.0; Cb[j] = L.Cv[j]; }
    Cb[6] = L.Dv;
#pragma unroll
    for (int j = 0; j < NC; ++j) b[j] = 0.0;
#pragma unroll 1
    for (int k = 0; k < NP; ++k) {
      double Hvk;
      pred_step(L.a, Cb, S, P, Hvk, row);
      const double g = cf.v_max - (rowdot(row, dx) + L.bv * 1.0);
      pb[(T::GAM + 4 * NC + k) * n + c] = g;
      pb[(T::HV + k) * n + c] = Hvk;
#pragma unroll
      for (int j = NC - 1; j > 0; --j) b[j] = b[j - 1];
      b[0] = Hvk;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NC; ++j) acc = acc + b[j] * DU[j];
      if (acc - g > 0) nv++;
      if (acc - g > 1e-9) nviol++;
    }
  }
  {  // -G_e rows: predMat(Cphi, Dphi), gamma = -phise_min + (Phi_e*dx + bphi)
    double S[6], P[6], Cb[7], row[7], b[NC];
#pragma unroll
    for (int j = 0; j < 6; ++j) { S[j] = 0.0; P[j] = 1.0; Cb[j] = L.Cphi[j]; }
    Cb[6] = L.Dphi;
#pragma unroll
    for (int j = 0; j < NC; ++j) b[j] = -0.0;
#pragma unroll 1
    for (int k = 0; k < NP; ++k) {
      double Hek;
      pred_step(L.a, Cb, S, P, Hek, row);
      const double g = -cf.phise_min + (rowdot(row, dx) + L.bphi * 1.0);
      pb[(T::GAM + 4 * NC + NP + k) * n + c] = g;
      pb[(T::HE + k) * n + c] = Hek;
#pragma unroll
      for (int j = NC - 1; j > 0; --j) b[j] = b[j - 1];
      b[0] = -Hek;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NC; ++j) acc = acc + b[j] * DU[j];
      if (acc - g > 0) nv++;
      if (acc - g > 1e-9) nviol++;
    }
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {  // G_soc rows
    const double g = gs[k];
    pb[(T::GAM + 4 * NC + 2 * NP + k) * n + c] = g;
    pb[(T::HS + k) * n + c] = Hs[k];
    pb[(T::ERR + k) * n + c] = e[k];
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + (j <= k ? Hs[k - j] : 0.0) * DU[j];
    if (acc - g > 0) nv++;
    if (acc - g > 1e-9) nviol++;
  }
  pb[T::RU * n + c] = Ru;
  pb[T::UK1 * n + c] = uk_1;
  if (nv == 0) {  // iterMPC.m:66-95 without hildreth.m: J_fin = J_unc (same DU)
    const double uk = DU[0] + uk_1;
    s.uk_1[c] = uk;
    if (s.J_fin) { s.J_fin[c] = J_unc; s.nviol[c] = nviol; }
    cost_out(io, c, J_unc, nviol, norm_du<NC>(DU));
    if (io.uk_out) io.uk_out[c] = uk;
    if (io.nexec) io.nexec[c] = 0;
    if (fused) {
      s.uk[c] = uk;
      if (io.u) io.u[c] = uk;
    }
    return;
  }
  s.hflag[c] = 1;
}

// M(i, :) of row i as a vector (constant rows by mconst, Toeplitz rows from H)
template <int NP, int NC>
__device__ __forceinline__ void mrow_vec(int i, const double *Hb, double b[NC]) {
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    if (i < 4 * NC) {
      b[k] = mconst<NC>(i, k);
    } else {
      const int blk = (i - 4 * NC) / NP, r = (i - 4 * NC) % NP;
      const double h = k <= r ? Hb[r - k] : 0.0;
      b[k] = blk == 1 ? -h : h;
    }
  }
}

// One row of k_hild_prep: K_i = M(i,:)*(E\F) + gamma_i, and for a distinct row X(:,u) =
// E\M(i,:)' and H_ii (also stored for the negated copy at i + NC when dup)
template <int NP, int NC>
__device__ __forceinline__ void prep_row(const KWide &w, const double *pb, int64_t n, int64_t c, int i, bool neg,
                                         int u, bool dup, const double R[NC][NC], const double y[NC],
                                         const double b[NC], double gam, bool &fin, double *xt, bool act) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  double kk = 0.0;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    kk = kk + b[k] * y[k];
    fin = fin && isfinite(b[k]);
  }
  if (act) w.K[(size_t)c * NCON + i] = kk + gam;
  if (neg || MPCEKF_WIDE_XPRO) return;  // H_ii of -b equals that of b (stored with the b row)
  double x[NC];
  chol_apply<NC>(R, b, x);
  double h = 0.0;
  const int l = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    h = h + b[k] * x[k];
    fin = fin && isfinite(x[k]);
    xt[l * (NC + 1) + k] = x[k];  // odd stride: fewer bank conflicts
  }
  if (act) {
    w.hii[(size_t)c * NCON + i] = h;
    if (dup) w.hii[(size_t)c * NCON + i + NC] = h;
  }
  // X(:, u) of the wave's 64 cells is one contiguous [64][NC] span of w.X: written back
  // from the LDS tile as 64 consecutive doubles per store (lane-per-cell stores of x[k]
  // hit 64 lines per instruction), only the active cells' entries
  __syncthreads();  // one wave per block
  const int64_t c0 = (int64_t)blockIdx.x * blockDim.x;
  const uint64_t am = __ballot(act);
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int e = j * 64 + l, cl = e / NC;
    if ((am >> cl) & 1) w.X[((size_t)u * n + c0) * NC + e] = xt[cl * (NC + 1) + e % NC];
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// k_hild_prep: hildreth.m:28-29 for the cells that run it (hflag == 1)
// ---------------------------------------------------------------------------
// hflag after: 1 = k_hild_wide, 2 = exact path with X/K/H_ii ready, 3 = exact path
// that must build them (E not SPD: MATLAB's \ falls back to LU), 4 (XPRO) = exact path
// that builds X/H_ii from the stored R (K ready).
template <int NP, int NC>
__global__ void __launch_bounds__(64) k_hild_prep(const KState s, const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  __shared__ double xt[64 * (NC + 1)];  // the wave's X(:, u) tile (one wave per block)
  const int64_t n = s.n;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool act = c < n && s.hflag[c] == 1;
  if (!__ballot(act)) return;  // uniform: every lane of the wave takes part in the tile stores
  const int64_t cr = act ? c : (int64_t)blockIdx.x * blockDim.x;  // inactive lanes read a valid cell
  const double *pb = w.prob;
  double E[NC][NC], R[NC][NC], F[NC], y[NC];
  load_E<NP, NC>(pb, n, cr, E);
  if (!chol_n<NC>(E, R) && act) {
    s.hflag[c] = 3;
    act = false;
  }
  if (MPCEKF_WIDE_XPRO && act) {
    int e = 0;
#pragma unroll
    for (int a = 0; a < NC; ++a)
#pragma unroll
      for (int b = a; b < NC; ++b) w.R[(size_t)(e++) * n + c] = R[a][b];
  }
#pragma unroll
  for (int a = 0; a < NC; ++a) F[a] = pb[(T::F + a) * n + cr];
  chol_apply<NC>(R, F, y);
  // The row loops stay rolled (fully unrolled the kernel was ~45k straight-line
  // instructions; rolled or unrolled by 2 or 4 it measured the same, ~0.40 ms per step
  // at configs[4]).  Row i's M(i, :) is built at run time (mconst / the Toeplitz shift
  // register), with mrow_vec's values and the same arithmetic per row.
  bool fin = true;
  // gamma_i (and the next Toeplitz entry) are loaded one row ahead: vmcnt counts stores
  // too, so a load issued after a row's stores would wait for their completion
  double gam = pb[T::GAM * n + cr];
#pragma unroll PREP_UNROLL
  for (int i = 0; i < 4 * NC; ++i) {  // [Cu; -Cu; I; -I]
    const double gi = gam;
    gam = pb[(T::GAM + i + 1) * n + cr];
    double b[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) b[k] = mconst<NC>(i, k);
    prep_row<NP, NC>(w, pb, n, cr, i, xneg<NC>(i), xslot<NP, NC>(i), i < NC || (i >= 2 * NC && i < 3 * NC), R, y, b,
                     gi, fin, xt, act);
  }
  double hn = pb[T::HV * n + cr];
#pragma unroll 1
  for (int blk = 0; blk < 3; ++blk) {  // [G_v; -G_e; G_soc] (constraintsMPC.m:44-80)
    // row r of a block: M(r, k) = +-H(r - k) for k <= r, +-0 beyond (mrow_vec's -h of
    // h = 0.0 in the negated block); row r + 1 shifts row r right by one
    double b[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) b[k] = blk == 1 ? -0.0 : 0.0;
#pragma unroll PREP_UNROLL
    for (int r = 0; r < NP; ++r) {
#pragma unroll
      for (int k = NC - 1; k > 0; --k) b[k] = b[k - 1];
      const double h = hn;
      b[0] = blk == 1 ? -h : h;
      const int i = 4 * NC + blk * NP + r;
      const double gi = gam;
      hn = pb[(T::HV + blk * NP + r + 1) * n + cr];  // HV + 3 NP is GAM: in the record
      gam = pb[(T::GAM + i + 1) * n + cr];          // GAM + NCON is ERR: in the record
      prep_row<NP, NC>(w, pb, n, cr, i, false, i - 2 * NC, false, R, y, b, gi, fin, xt, act);
    }
  }
  // a non-finite M entry (XPRO: X is checked by k_hild_wide): the exact path, which with
  // XPRO builds X and H_ii from R first (hflag 4)
  if (act && !fin) s.hflag[c] = MPCEKF_WIDE_XPRO ? 4 : 2;
}

// ---------------------------------------------------------------------------
// k_hild_bin / k_hild_sort: the fast-path cells listed by predicted sweeps
// ---------------------------------------------------------------------------
// k_hild_wide runs 8 cells per wave and a wave lasts as long as its slowest cell; a
// cell's count changes little from one control step to the next, so listing cells by
// last step's count (longest first) puts cells of like length in one wave.  The order
// only decides which group runs which cell: each cell's sweeps are the same operations
// whichever group runs them, so the results are the bits of any other order.
// A 1024-thread block takes LIST_CPB cells, bins them in LDS and adds its bin totals to
// the global counters with one atomic per nonzero bin (per-cell global atomics on the
// few hot bins serialised at the L2: ~0.5 ms a step).  LIST = false: the
// histogram; LIST = true: the list, each cell's slot = its block's range in the bin
// (reserved on the offsets k_hild_sort left) + its rank in the block.
constexpr int LIST_CPB = 4096;
template <bool LIST>
__global__ void __launch_bounds__(1024) k_hild_bin(const KCfg cf, const KState s, const KWide w) {
  __shared__ int lh[SWEEP_BINS], gb[SWEEP_BINS];
  const int t = threadIdx.x;
  if (t < SWEEP_BINS) lh[t] = 0;
  __syncthreads();
  constexpr int CPT = LIST_CPB / 1024;
  int bin[CPT], rank[CPT];
  const int64_t c0 = (int64_t)blockIdx.x * LIST_CPB + t;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int64_t c = c0 + j * 1024;
    const bool act = c < s.n && s.hflag[c] == 1;
    bin[j] = act ? sweep_bin(w.it[c], cf.max_hild) : -1;
    rank[j] = act ? atomicAdd(&lh[bin[j]], 1) : 0;
  }
  __syncthreads();
  int *ctr = LIST ? w.hist + SWEEP_BINS : w.hist;
  if (t < SWEEP_BINS) gb[t] = lh[t] ? atomicAdd(&ctr[t], lh[t]) : 0;
  if (!LIST) return;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < CPT; ++j)
    if (bin[j] >= 0) w.list[gb[bin[j]] + rank[j]] = (int)(c0 + j * 1024);
}

__global__ void __launch_bounds__(64) k_hild_sort(const KWide w) {
  if (threadIdx.x != 0) return;
  int acc = 0;
  for (int b = SWEEP_BINS - 1; b >= 0; --b) {  // descending: longest first
    w.hist[SWEEP_BINS + b] = acc;
    acc += w.hist[b];
    w.hist[b] = 0;  // ready for the next step's k_hild_bin<false>
  }
  w.q[0] = acc;
}


// ---------------------------------------------------------------------------
// k_hild_wide: hildreth.m:32-42 with an 8-lane group per cell
// ---------------------------------------------------------------------------
// A 16-lane DPP row holds two cells (lanes 0-7 and 8-15); every DPP pattern below stays
// inside its 8-lane group.  64-bit DPP exists only for row_newbcast, so a double moves as
// two v_mov_b32_dpp.
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// the DPP move into the lanes of the banks in BANK only; the other lanes keep `old`
template <int CTRL, int BANK>
__device__ __forceinline__ double dpp64_into(double old, double v) {
  const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, 0xF, BANK, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, 0xF, BANK, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// Sum over the 8 lanes of a group as the pairwise tree of hild_row_t: each level adds the
// partner's partial sum (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror); both partners
// add the same two values, so every lane ends with the same bits.
__device__ __forceinline__ double tree8(double a) {
  a = a + dpp64<0xB1>(a);
  a = a + dpp64<0x4E>(a);
  a = a + dpp64<0x141>(a);
  return a;
}
// lane J's value in every lane of its 8-lane group: quad_perm [J%4 x4] gives each quad its
// lane J%4, then the quad that holds lane J is copied into the other (row_shr:4 into banks
// 1 and 3 for J < 4, row_shl:4 into banks 0 and 2 for J >= 4)
template <int J>
__device__ __forceinline__ double bcast8(double v) {
  const double q = dpp64<(J & 3) * 0x55>(v);
  return J < 4 ? dpp64_into<0x114, 0xA>(q, q) : dpp64_into<0x104, 0x5>(q, q);
}
__device__ __forceinline__ double bcast8(double v, int j) {  // j a constant after unrolling
  switch (j) {
    case 0: return bcast8<0>(v);
    case 1: return bcast8<1>(v);
    case 2: return bcast8<2>(v);
    case 3: return bcast8<3>(v);
    case 4: return bcast8<4>(v);
    case 5: return bcast8<5>(v);
    case 6: return bcast8<6>(v);
    default: return bcast8<7>(v);
  }
}

// The row term b_k of hild_row_t for lane k (columns k and k + 8): a_0 = fma(M_i0, v_0, K_i),
// a_k = M_ik v_k, as fma(M_ik, v_k, kz) with kz = K_i in lane 0 and +0 elsewhere (fma(m, v, +0)
// differs from m*v only in the sign of a zero product, which cannot reach t); then
// b_k = fma(M_i,k+8, v_k+8, a_k).  Constant rows (M entries +-1 / +-0) become an add or a
// select.  A lane whose column k + 8 does not exist holds a stray v1 (see x1_to_lanes01)
// and reads a zero M entry for it, or is not selected.
template <int NP, int NC>
__device__ __forceinline__ double row_term8(int i, int k, double v0, double v1, double kz, double m0, double m1) {
  if (i < NC) {  // Cu row i: ones in columns 0..i
    double a = k <= i ? v0 + kz : kz;
    if (i >= 8) a = (k + 8 <= i && k + 8 < NC) ? a + v1 : a;
    return a;
  }
  if (i < 2 * NC) {  // -Cu
    const int r = i - NC;
    double a = k <= r ? kz - v0 : kz;
    if (r >= 8) a = (k + 8 <= r && k + 8 < NC) ? a - v1 : a;
    return a;
  }
  const int blk = (i - 4 * NC) / NP, r = (i - 4 * NC) % NP;
  double a = blk == 1 ? __builtin_fma(-m0, v0, kz) : __builtin_fma(m0, v0, kz);
  if (r >= 8 && NC > 8) a = blk == 1 ? __builtin_fma(-m1, v1, a) : __builtin_fma(m1, v1, a);
  return a;
}
// The I / -I rows (one M entry, +-1 in column j): the tree of hild_row_t adds K_i and +-v_j
// to zeros only, which is exact, so t = K_i +- v_j in one rounding (the sign of a zero t
// aside, which cannot reach lambda: min(t (1/H_ii), lambda_i) is then +-0 or lambda_i, so
// lambda_i - min(..) and the step's effect on v are the same for either sign).  v_j comes from lane j % 8 of the group (v0 for j < 8,
// v1 above) by bcast8; K_i is read in every lane.
template <int NC>
__device__ __forceinline__ constexpr bool unit_row(int i) {
  return i >= 2 * NC && i < 4 * NC;
}
template <int NC>
__device__ __forceinline__ double unit_t(int i, double v0, double v1, double K) {
  static_assert(NC <= 16, "two columns per lane of an 8-lane group");
  const int j = (i - 2 * NC) % NC;
  const double vj = j < 8 ? bcast8(v0, j) : bcast8(v1, j - 8);
  return i < 3 * NC ? K + vj : K - vj;
}
// Rows whose nonzero terms sit in lanes 0 .. 2^L - 1 only (after folding column k + 8 into
// lane k): L = 0 (one term: the first Cu / -Cu row, the first row of each Toeplitz block)
// broadcasts lane 0, L = 1 adds one level first; otherwise the full tree, whose extra levels
// would add exact zeros (the sign of a zero t aside, as for unit_t).
template <int NP, int NC>
__device__ __forceinline__ constexpr int row_levels8(int i) {
  const int nz = i < NC ? i + 1 : i < 2 * NC ? i - NC + 1 : ((i - 4 * NC) % NP + 1 < NC ? (i - 4 * NC) % NP + 1 : NC);
  const int lanes = nz < 8 ? nz : 8;
  return lanes <= 1 ? 0 : lanes <= 2 ? 1 : 3;
}
__device__ __forceinline__ double tree_rows8(int L, double a) {  // L a constant after unrolling
  if (L >= 3) return tree8(a);
  if (L >= 1) a = a + dpp64<0xB1>(a);
  return bcast8<0>(a);
}
// lane k's M entry of Toeplitz row i for column col (0 for the constant rows, which
// row_term8 builds); mp points at the block-0 entry of row 0 for this lane's column
template <int NP, int NC>
__device__ __forceinline__ double row_m(int i, const double *mp) {
  if (i < 4 * NC) return 0.0;
  const int blk = (i - 4 * NC) / NP, r = (i - 4 * NC) % NP;
  return mp[blk * W<NP, NC>::HPW + r];
}

// X's columns 8 .. Nc-1 (lanes 0 .. Nc-9 of a group use them) are held spread over the
// group: row u's pair sits in lanes 2q, 2q + 1 (q = u % 4) at register slot u / 4, and is
// moved into lanes 0, 1 by one row_shl:2q when row u runs.  80 more doubles per lane for
// column k + 8 did not fit beside column k's 80.  The other lanes receive the values of
// lanes further up the group, or +0 where the shift reads past the 16-lane DPP row
// (bound_ctrl: a defined zero, not a stale register), which every use masks: their M
// entries for columns >= 8 are read from the zero row, and the Cu rows select on the lane.
template <int CTRL>
__device__ __forceinline__ double dpp64_zf(double v) {  // invalid source lanes read +0
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
template <int Q>
__device__ __forceinline__ double x1_to_lanes01(double v) {
  if constexpr (Q == 0) return v;
  else return dpp64_zf<0x100 + 2 * Q>(v);  // row_shl:2Q
}
__device__ __forceinline__ double x1_to_lanes01(double v, int q) {  // q a constant after unrolling
  switch (q) {
    case 0: return x1_to_lanes01<0>(v);
    case 1: return x1_to_lanes01<1>(v);
    case 2: return x1_to_lanes01<2>(v);
    default: return x1_to_lanes01<3>(v);
  }
}

template <int NP, int NC>
__global__ void __launch_bounds__(128, 1) k_hild_wide(const KCfg cf, const KState s, const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON, HPW = T::HPW, LN = T::LANES;
  static_assert(LN == 8 && NC > LN && T::BLOCK == 128, "8-lane groups with columns >= 8 (Nc = 10); the launch bounds");
  extern __shared__ double lds[];
  double *zero = lds;  // NCON zeros: lanes that add no K_i read these
  const int g = threadIdx.x / LN, k = threadIdx.x % LN;
  const int64_t n = s.n, slot = (int64_t)blockIdx.x * T::GROUPS + g;
  static_assert(T::ZERO_LDS % 2 == 0 && T::CELL_LDS % 2 == 0, "16-byte aligned (H_ii, 1/H_ii) pairs");
  double *base = lds + T::ZERO_LDS + g * T::CELL_LDS;
  double2 *hr = reinterpret_cast<double2 *>(base);  // (H_ii, 1/H_ii)
  double *lam = base + 2 * NCON, *Kl = lam + NCON, *hp = Kl + NCON;
  static_assert(4 * NCON + 3 * HPW <= T::CELL_LDS &&
                    2 * (T::ZERO_LDS + T::GROUPS * T::CELL_LDS + T::WAVES * T::JUNK) * 8 <= 160 * 1024,
                "two blocks per CU");
  for (int i = threadIdx.x; i < NCON; i += blockDim.x) zero[i] = 0.0;
  if (MPCEKF_WIDE_XPRO && (int64_t)blockIdx.x * T::GROUPS >= w.q[0]) return;  // block-uniform: nothing listed
  const bool act = slot < w.q[0];            // k_hild_sort's count
  const int64_t c = act ? w.list[slot] : 0;  // cells in k_hild_bin<true>'s order
  bool ok = true;
  static_assert(NC <= LN + 2 && T::NX_ROWS % LN == 0, "columns >= 8 spread as pairs over 4 lane pairs");
  double X0[T::NX_ROWS], X1[T::NX_ROWS / 4];
#if MPCEKF_WIDE_XPRO
  // hildreth.m:28's X(:,i) = E\M(i,:)' and H_ii = M(i,:)*X(:,i) for the group's cell, from
  // k_hild_prep's R = chol(E): lane k solves the distinct rows u = 8j + k (chol_apply, the
  // arithmetic k_hild_prep would use), and the group transposes each chunk of 8 solutions
  // through LDS so that lane k keeps columns k (and k + 8 spread over the lane pairs) of
  // every row.  X never goes through HBM.  Inactive groups of the block run it on cell 0's
  // data (results unused) so that every lane reaches the barriers.
  for (int j = k; j < 3 * HPW; j += LN) {
    const int b = j / HPW, q = j % HPW;
    hp[j] = q < NC - 1 ? 0.0 : w.prob[(T::HV + b * NP + q - (NC - 1)) * n + c];
  }
  double R[NC][NC];
  {
    int e = 0;
#pragma unroll
    for (int a = 0; a < NC; ++a)
#pragma unroll
      for (int b = a; b < NC; ++b) R[a][b] = w.R[(size_t)(e++) * n + c];
  }
  __syncthreads();                 // hp
  double *xb = lam;                // a chunk's 8 solutions [8][NC]; lam / K are filled after
#pragma unroll
  for (int j = 0; j < T::NX_ROWS / LN; ++j) {
    const int u = LN * j + k;
    // M(i,:) of the distinct row u, as mrow_vec / k_hild_prep build it: the Cu rows, the I
    // rows, then the Toeplitz blocks (+-H(r - m), +-0 beyond r)
    const int tu = u >= 2 * NC ? u - 2 * NC : 0, blk = tu / NP, r = tu % NP;
    double b[NC], x[NC];
#pragma unroll
    for (int m = 0; m < NC; ++m) {
      const double hv = hp[blk * HPW + (NC - 1) + r - m];
      b[m] = u < NC ? (m <= u ? 1.0 : 0.0) : u < 2 * NC ? (u - NC == m ? 1.0 : 0.0) : (blk == 1 ? -hv : hv);
    }
    chol_apply<NC>(R, b, x);
    double h = 0.0;
#pragma unroll
    for (int m = 0; m < NC; ++m) {
      h = h + b[m] * x[m];
      ok = ok && isfinite(x[m]);
      xb[k * NC + m] = x[m];
    }
    const int i = u < NC ? u : u < 2 * NC ? u + NC : u + 2 * NC;  // constraint row (+ NC: its negated copy)
    ok = ok && hild_rok(h);                          // hild_step's reciprocal form for every row
    const double2 hh = make_double2(h, 1.0 / h);     // the oracle's 1.0 / hii (IEEE)
    hr[i] = hh;
    if (u < 2 * NC) hr[i + NC] = hh;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < LN; ++q) X0[LN * j + q] = xb[q * NC + k];
    X1[2 * j] = xb[(k >> 1) * NC + LN + (k & 1)];
    X1[2 * j + 1] = xb[(4 + (k >> 1)) * NC + LN + (k & 1)];
    __syncthreads();
  }
  if (act) {
    for (int i = k; i < NCON; i += LN) {
      const double li = s.lam[(size_t)i * n + c];
      ok = ok && isfinite(li);
      lam[i] = li;
      Kl[i] = w.K[(size_t)c * NCON + i];
    }
  }
#else
  if (act) {
    for (int i = k; i < NCON; i += LN) {
      const double li = s.lam[(size_t)i * n + c];
      const double hii = w.hii[(size_t)c * NCON + i];
      ok = ok && isfinite(li) && hild_rok(hii);
      lam[i] = li;
      Kl[i] = w.K[(size_t)c * NCON + i];
      hr[i] = make_double2(hii, 1.0 / hii);
    }
    for (int j = k; j < 3 * HPW; j += LN) {
      const int b = j / HPW, q = j % HPW;
      hp[j] = q < NC - 1 ? 0.0 : w.prob[(T::HV + b * NP + q - (NC - 1)) * n + c];
    }
  }
#endif
  __syncthreads();
  if (!act) return;
  const int gshift = LN * (g % (64 / LN));
  constexpr int SLOW = MPCEKF_WIDE_XPRO ? 4 : 2;  // the exact path (4: it builds X / H_ii first)
  if ((__ballot(!ok) >> gshift) & 0xFFull) {  // outside the fast form's domain
    if (k == 0) s.hflag[c] = SLOW;
    return;
  }
  const double *kp = k == 0 ? Kl : zero;
  // lanes whose column does not exist read column Nc-1's entry (a broadcast, no bank of
  // their own): their v is +0 for good (X there is 0 and lambda >= 0), so the term is +-0
  const int col0 = k < NC ? k : NC - 1;
  const double *mp0 = hp + (NC - 1) - col0;
  const double *mp1 = k + LN < NC ? hp + (NC - 1) - (k + LN) : zero;  // zero: the stray lanes
  // lambda_i store: lane k = 0 writes lam[i]; the other lanes write their own slot of a
  // per-wave sink (8 lanes storing one address serialise in one LDS bank, and an
  // exec-masked store splits the wave's control flow inside the row)
  double *lst = lam;
  if (k != 0) lst = lds + T::ZERO_LDS + T::GROUPS * T::CELL_LDS + (threadIdx.x >> 6) * T::JUNK + (threadIdx.x & 63);
#if !MPCEKF_WIDE_XPRO
#pragma unroll
  for (int u = 0; u < T::NX_ROWS; ++u) X0[u] = k < NC ? w.X[((size_t)u * n + c) * NC + k] : 0.0;
#pragma unroll
  for (int sl = 0; sl < T::NX_ROWS / 4; ++sl) {
    const int u = 4 * sl + (k >> 1), col = LN + (k & 1);
    X1[sl] = col < NC ? w.X[((size_t)u * n + c) * NC + col] : 0.0;
  }
#endif
  // X(:, i) of constraint row i for lane k's two columns (the -Cu / -I rows negated)
  auto xrow = [&](int i, double &x0, double &x1) {
    const int u = xslot<NP, NC>(i);
    const double a = X0[u], b = x1_to_lanes01(X1[u / 4], u % 4);
    x0 = xneg<NC>(i) ? -a : a;
    x1 = xneg<NC>(i) ? -b : b;
  };
  // lane k's M entries of row i (columns k and k + 8; the constant rows build theirs)
  auto mrow = [&](int i, double &m0, double &m1) {
    m0 = row_m<NP, NC>(i, mp0);
    m1 = (i >= 4 * NC && (i - 4 * NC) % NP >= 8 && NC > 8) ? row_m<NP, NC>(i, mp1) : 0.0;
  };
  // K_i + M(i,:)*v as hild_row_t's lane tree (kz = K_i in lane 0, +0 elsewhere; K_i in
  // every lane of a unit row)
  auto rowT = [&](int i, double a0, double a1, double kz, double m0, double m1) {
    return unit_row<NC>(i) ? unit_t<NC>(i, a0, a1, kz)
                           : tree_rows8(row_levels8<NP, NC>(i), row_term8<NP, NC>(i, k, a0, a1, kz, m0, m1));
  };
  const double tol = cf.hild_tol;
  const int maxIter = cf.max_hild;
  // v = X*lambda at the start of a sweep (orc hild_v: fma from +0 in ascending j).  The
  // first one is summed here from the warm start; each sweep then accumulates the next
  // sweep's (u0, u1) row by row from lambda_j's final value of this sweep, which is the same
  // sequence of fmas on the same operands as summing after the sweep, without a second
  // pass over X and lambda.
  double v0 = 0.0, v1 = 0.0;
#pragma unroll
  for (int j = 0; j < NCON; ++j) {
    if (j % 4 == 0) asm volatile("" ::: "memory");  // no hoisting of every row's loads
    double x0, x1;
    xrow(j, x0, x1);
    const double lj = lam[j];
    v0 = __builtin_fma(x0, lj, v0);
    v1 = __builtin_fma(x1, lj, v1);
  }
  int it;
  bool slow = false;
  for (it = 1; it <= maxIter; ++it) {
    // K_i, (H_ii, 1/H_ii) and the M entries are re-read from LDS every sweep
    asm volatile("" ::: "memory");
    double u0 = 0.0, u1 = 0.0;  // the next sweep's v
    // hildreth.m:39's stop test as a wave mask (|d| < tol on every row; a NaN d is "not
    // converged", as in orc_hildreth; the 8 lanes of a group compute the same d)
    uint64_t convm = ~0ull;
    // A row's LDS operands are read PF rows ahead: the compiler pulls a row's first
    // operations up into the row before, and a one-row distance then left the reads ~20
    // instructions to land (PF = 2: 3.70 -> 3.59 ms per step at configs[4]).
    constexpr int PF = MPCEKF_WIDE_PF, RING = PF + 1;
    struct Ops {
      double kz, m0, m1, li;
      double2 h;
    } q[RING];
    auto load_ops = [&](int r) {
      Ops &o = q[r % RING];
      o.kz = unit_row<NC>(r) ? Kl[r] : kp[r];
      mrow(r, o.m0, o.m1);
      o.li = lam[r];
      o.h = hr[r];
    };
#pragma unroll
    for (int r = 0; r < PF && r < NCON; ++r) load_ops(r);
#pragma unroll
    for (int i = 0; i < NCON; ++i) {
      asm volatile("" ::: "memory");  // loads stay in their rows, not all at the sweep start
      if (i + PF < NCON) load_ops(i + PF);
      const Ops &o = q[i % RING];
      const double t = rowT(i, v0, v1, o.kz, o.m0, o.m1);
      const double li = o.li;
      const double2 h = o.h;
      // hild_step's reciprocal form: m = min(t / H_ii, lambda_i) with t (1/H_ii), the step -m,
      // lambda_i - m: every H_ii is in its domain (checked at the staging) and lambda_i finite
      // while v is (a zero H(0) row's 1/H_ii = +-inf gives x / +-0 by IEEE)
      const double m = fmin_q(t * h.y, li);   // fmin without the canonicalising max of lambda_i
      const double nl = li - m;
      convm &= __ballot(fabs(m) < tol);
      lst[i] = nl;
      double x0, x1;
      xrow(i, x0, x1);
      v0 = __builtin_fma(-x0, m, v0);   // fma(x, d, v) with the step d = -m
      v1 = __builtin_fma(-x1, m, v1);
      u0 = __builtin_fma(x0, nl, u0);
      u1 = __builtin_fma(x1, nl, u1);
      // every accumulation finishes in its row: left alone, the compiler sank the ones not
      // needed before the sweep end (u, the stop flag) and held every row's lambda and step
      // live across the sweep
      asm volatile("" : "+v"(u0), "+v"(u1), "+v"(v1), "+s"(convm));
    }
    // a non-finite v (a zero-diagonal row going to or from +inf): the exact path redoes
    // this cell from its warm start, still in s.lam (every sweep before was bit-identical
    // to the exact form)
    const bool bad = !(isfinite(v0) && isfinite(v1));
    if ((__ballot(bad) >> gshift) & 0xFFull) {
      slow = true;
      break;
    }
    if ((convm >> gshift) & 1ull) break;
    v0 = u0;
    v1 = u1;
  }
  if (slow) {
    if (k == 0) s.hflag[c] = SLOW;
    return;
  }
  if (it > maxIter) it = maxIter;
  for (int i = k; i < NCON; i += LN) s.lam[(size_t)i * n + c] = lam[i];
  if (k == 0) w.it[c] = it;
}

// ---------------------------------------------------------------------------
// k_hild_wide_slow: orc_hildreth with every rule, lane per cell (hflag 2 / 3 / 4)
// ---------------------------------------------------------------------------
template <int NP, int NC>
__device__ __forceinline__ double xval_g(const double *X, int64_t n, int64_t c, int i, int k) {
  const double x = X[((size_t)xslot<NP, NC>(i) * n + c) * NC + k];
  return xneg<NC>(i) ? -x : x;
}

template <int NP, int NC>
__device__ __forceinline__ double mval_rt(const double *Hall, int i, int k) {  // runtime i
  if (i < 4 * NC) {
    if (i < NC) return k <= i ? 1.0 : 0.0;
    if (i < 2 * NC) return -((k <= i - NC) ? 1.0 : 0.0);
    if (i < 3 * NC) return (i - 2 * NC) == k ? 1.0 : 0.0;
    return -((i - 3 * NC) == k ? 1.0 : 0.0);
  }
  const int blk = (i - 4 * NC) / NP, r = (i - 4 * NC) % NP;
  const double h = k <= r ? Hall[blk * NP + r - k] : 0.0;
  return blk == 1 ? -h : h;
}

template <int NP, int NC>
__device__ __forceinline__ double row_t_rt(const double *Hall, int i, const double v[NC], double Ki) {
  if (NC <= 2) {
    double t = Ki;
#pragma unroll
    for (int k = 0; k < NC; ++k) t = __builtin_fma(mval_rt<NP, NC>(Hall, i, k), v[k], t);
    return t;
  }
  double b[8];  // orc hild_row_t's 8-lane form
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double a = k == 0 ? __builtin_fma(mval_rt<NP, NC>(Hall, i, 0), v[0], Ki)
                            : (k < NC ? mval_rt<NP, NC>(Hall, i, k) * v[k] : 0.0);
    b[k] = k + 8 < NC ? __builtin_fma(mval_rt<NP, NC>(Hall, i, k + 8 < NC ? k + 8 : 0), v[k + 8 < NC ? k + 8 : 0], a) : a;
  }
#pragma unroll
  for (int wd = 1; wd < 8; wd *= 2)
#pragma unroll
    for (int k = 0; k < 8; k += 2 * wd) b[k] = b[k] + b[k + wd];
  return b[0];
}

template <int NP, int NC>
__device__ __forceinline__ void hild_v_g(const double *X, int64_t n, int64_t c, const double *lam, double v[NC]) {
  constexpr int NCON = W<NP, NC>::NCON;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    double a = 0.0;
#pragma unroll 1
    for (int j = 0; j < NCON; ++j) a = __builtin_fma(xval_g<NP, NC>(X, n, c, j, k), lam[(size_t)j * n + c], a);
    v[k] = a;
  }
}

template <int NP, int NC>
__global__ void __launch_bounds__(64) k_hild_wide_slow(const KCfg cf, const KState s, const KWide w) {
  using T = W<NP, NC>;
  constexpr int NCON = T::NCON;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  if (c >= n || s.hflag[c] < 2) return;
  const double *pb = w.prob;
  double Hall[3 * NP];
#pragma unroll
  for (int r = 0; r < 3 * NP; ++r) Hall[r] = pb[(T::HV + r) * n + c];
  bool fin = true;
  if (s.hflag[c] == 3) {  // E not SPD: X(:,i) = E\M(i,:)' by LU (MATLAB's \ fallback)
    double E[NC][NC], F[NC], y[NC];
    load_E<NP, NC>(pb, n, c, E);
#pragma unroll
    for (int a = 0; a < NC; ++a) F[a] = pb[(T::F + a) * n + c];
    lu_solve_n<NC>(E, F, y);
#pragma unroll 1
    for (int i = 0; i < NCON; ++i) {
      double b[NC], x[NC];
      double kk = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        b[k] = mval_rt<NP, NC>(Hall, i, k);
        kk = kk + b[k] * y[k];
      }
      w.K[(size_t)c * NCON + i] = kk + pb[(T::GAM + i) * n + c];
      lu_solve_n<NC>(E, b, x);
      double h = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) h = h + b[k] * x[k];
      w.hii[(size_t)c * NCON + i] = h;
      if (!xneg<NC>(i)) {
#pragma unroll
        for (int k = 0; k < NC; ++k) w.X[((size_t)xslot<NP, NC>(i) * n + c) * NC + k] = x[k];
      }
    }
  } else if (s.hflag[c] == 4) {  // X(:,i) and H_ii from k_hild_prep's R, as k_hild_prep would build them
    double R[NC][NC];
    int e = 0;
#pragma unroll
    for (int a = 0; a < NC; ++a)
#pragma unroll
      for (int b = a; b < NC; ++b) R[a][b] = w.R[(size_t)(e++) * n + c];
#pragma unroll 1
    for (int i = 0; i < NCON; ++i) {
      if (xneg<NC>(i)) continue;  // H_ii of -b is stored with the b row
      double b[NC], x[NC];
#pragma unroll
      for (int k = 0; k < NC; ++k) b[k] = mval_rt<NP, NC>(Hall, i, k);
      chol_apply<NC>(R, b, x);
      double h = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        h = h + b[k] * x[k];
        w.X[((size_t)xslot<NP, NC>(i) * n + c) * NC + k] = x[k];
      }
      w.hii[(size_t)c * NCON + i] = h;
      if (i < NC || (i >= 2 * NC && i < 3 * NC)) w.hii[(size_t)c * NCON + i + NC] = h;
    }
  }
#pragma unroll 1
  for (int i = 0; i < NCON; ++i)
#pragma unroll
    for (int k = 0; k < NC; ++k)
      fin = fin && isfinite(xval_g<NP, NC>(w.X, n, c, i, k)) && isfinite(mval_rt<NP, NC>(Hall, i, k));
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
      const double hii = w.hii[(size_t)c * NCON + i], Ki = w.K[(size_t)c * NCON + i];
      const double li = lam[(size_t)i * n + c];
      double nl, d;
      if (fin) {
        d = hild_step(row_t_rt<NP, NC>(Hall, i, v, Ki), hii, 1.0 / hii, li, nl);
      } else {  // dense H(i,:)*lambda, 4 interleaved partial sums (orc_hildreth)
        double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
        for (int j = 0; j < NCON; ++j) {
          double h = 0.0;
#pragma unroll
          for (int k = 0; k < NC; ++k) h = h + mval_rt<NP, NC>(Hall, i, k) * xval_g<NP, NC>(w.X, n, c, j, k);
          p[j & 3] = p[j & 3] + h * lam[(size_t)j * n + c];
        }
        const double sm = (p[0] + p[1]) + (p[2] + p[3]);
        const double wv = -((Ki + sm) - hii * li) / hii;
        nl = wv > 0 ? wv : 0.0;
        d = nl - li;
      }
      if (!(fabs(d) < tol)) conv = false;
      lam[(size_t)i * n + c] = nl;
      if (fin) {
        if (isfinite(d)) {
#pragma unroll
          for (int k = 0; k < NC; ++k) v[k] = __builtin_fma(xval_g<NP, NC>(w.X, n, c, i, k), d, v[k]);
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
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = s.n;
  if (c >= n || s.hflag[c] == 0) return;
  const double *pb = w.prob;
  // M'*lambda, summed over the rows in ascending order from +0 (orc_hildreth)
  double Mtl[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) Mtl[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 4 * NC; ++i) {
    if (i % 8 == 0) asm volatile("" ::: "memory");  // no hoisting of every row's loads
    const double li = s.lam[(size_t)i * n + c];
#pragma unroll
    for (int k = 0; k < NC; ++k) Mtl[k] = Mtl[k] + mconst<NC>(i, k) * li;
  }
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    double Hb[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) Hb[r] = pb[(T::HV + blk * NP + r) * n + c];
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      if (r % 8 == 0) asm volatile("" ::: "memory");
      const double li = s.lam[(size_t)(4 * NC + blk * NP + r) * n + c];
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        const double h = k <= r ? Hb[r - k] : 0.0;
        Mtl[k] = Mtl[k] + (blk == 1 ? -h : h) * li;
      }
    }
  }
  double mE[NC][NC], rhs[NC], DU[NC];
#pragma unroll
  for (int a = 0; a < NC; ++a) {
    rhs[a] = pb[(T::F + a) * n + c] + Mtl[a];
#pragma unroll
    for (int b = 0; b < NC; ++b) mE[a][b] = -pb[(T::E + a * NC + b) * n + c];
  }
  lu_solve_n<NC>(mE, rhs, DU);
  const double uk_1 = pb[T::UK1 * n + c];
  const double uk = DU[0] + uk_1;
  int nviol = 0;
#pragma unroll
  for (int i = 0; i < 4 * NC; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + mconst<NC>(i, j) * DU[j];
    if (acc - pb[(T::GAM + i) * n + c] > 1e-9) nviol++;
  }
  double Hs[NP];
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    double Hb[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) Hb[r] = pb[(T::HV + blk * NP + r) * n + c];
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const double h = j <= r ? Hb[r - j] : 0.0;
        acc = acc + (blk == 1 ? -h : h) * DU[j];
      }
      if (acc - pb[(T::GAM + 4 * NC + blk * NP + r) * n + c] > 1e-9) nviol++;
      if (blk == 2) Hs[r] = Hb[r];
    }
  }
  double e[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) e[i] = pb[(T::ERR + i) * n + c];
  s.uk_1[c] = uk;
  const double J_fin = mpc_cost<NP, NC>(Hs, e, pb[T::RU * n + c], DU);
  if (s.J_fin) {
    s.J_fin[c] = J_fin;
    s.nviol[c] = nviol;
  }
  cost_out(io, c, J_fin, nviol, norm_du<NC>(DU));
  if (io.uk_out) io.uk_out[c] = uk;
  if (io.nexec) io.nexec[c] = w.it[c];
  if (io.mode & MODE_FUSED) {
    s.uk[c] = uk;
    if (io.u) io.u[c] = uk;
  }
}

// GsocT*Gsoc and its sigma_min, as mpc_setup forms them for Csoc = [0 0 0 0 0 rr],
// Dsoc = 0 (EKFmatsHandler.m:43-45): the cache k_mpc_wide compares bitwise.
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
  return (W<NP, NC>::ZERO_LDS + W<NP, NC>::GROUPS * W<NP, NC>::CELL_LDS + W<NP, NC>::WAVES * W<NP, NC>::JUNK) *
         (int)sizeof(double);
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
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)k_hild_wide<WIDE_NP, WIDE_NC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_hild_prep<WIDE_NP, WIDE_NC>), dim3(grid(s.n, 64)), dim3(64), 0, st, s, w);
  hipLaunchKernelGGL(k_hild_bin<false>, dim3(grid(s.n, LIST_CPB)), dim3(1024), 0, st, c, s, w);
  hipLaunchKernelGGL(k_hild_sort, dim3(1), dim3(64), 0, st, w);
  hipLaunchKernelGGL(k_hild_bin<true>, dim3(grid(s.n, LIST_CPB)), dim3(1024), 0, st, c, s, w);
  hipLaunchKernelGGL((k_hild_wide<WIDE_NP, WIDE_NC>), dim3(grid(s.n, W<WIDE_NP, WIDE_NC>::GROUPS)),
                     dim3(W<WIDE_NP, WIDE_NC>::BLOCK), lds, st, c, s, w);
  hipLaunchKernelGGL((k_hild_wide_slow<WIDE_NP, WIDE_NC>), dim3(grid(s.n, 64)), dim3(64), 0, st, c, s, w);
  hipLaunchKernelGGL((k_mpc_wide_finish<WIDE_NP, WIDE_NC>), dim3(grid(s.n, 64)), dim3(64), 0, st, c, s, io, w);
  return (int)hipGetLastError();
}

int launch_cl_diag_wide(const KCfg &c, int64_t n, const double *lin, const double *uk1, double *poles, double *sv,
                        void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL((k_cl_diag<WIDE_NP, WIDE_NC>), dim3(grid(n, 64)), dim3(64), 0, (hipStream_t)stream, c, n, lin, uk1,
                     poles, sv);
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
