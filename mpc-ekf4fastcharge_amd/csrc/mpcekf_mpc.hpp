// mpcekf_mpc.hpp -- device-side MPC pieces shared by the kernel translation units,
// templated on the horizons (NP, NC): predMat.m, constraintsMPC.m and iterMPC.m.
// mpcekf_kernels.hip instantiates them for runMPC.m's Np = 5 / Nc = 2 (lane-per-cell
// fused step), mpcekf_wide.hip for Np = 20 / Nc = 10 (BASELINE.json configs[4]).
//
// Arithmetic follows oracle/mpcekf_oracle.c's defined order (sequential sums from +0,
// no contraction), so every instantiation is bit-identical to orc_mpc_step.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "mpcekf_eig.hpp"
#include "mpcekf_kernels.hpp"

#pragma clang fp contract(off)

namespace mk {

// Keep a value opaque to the optimiser (no code emitted).  Used to pin where a
// value is materialised (bounding register live ranges) and to stop the
// loop-invariant products of the Hildreth sweep from being hoisted into 529
// live registers.
__device__ __forceinline__ void launder(double &x) { asm volatile("" : "+v"(x)); }

// hildreth.m:35-36's update as oracle/mpcekf_oracle.c hild_step defines it (round 6): the
// step d = -min(t_i (1/H_ii), lambda_i) and lambda_i <- lambda_i - min(..), with the correctly
// rounded 1/H_ii formed once per solve, when H_ii is 0 or in [2^-1020, 2^1020] (hild_rok) and
// lambda_i is finite; the division form (w = fma(H_ii, lambda_i, -t_i) / H_ii, max(w, 0), the
// difference) otherwise.  fmin is v_min_f64 (a NaN operand yields the other: a NaN q leaves
// lambda_i = 0, as max(0, NaN) does); H_ii = +-0 gives 1/H_ii = +-inf, and t (+-inf) is x / +-0's
// inf / NaN by IEEE.  Returns d; nl = the new lambda_i.
__device__ __forceinline__ bool hild_rok(double h) {
  const double a = fabs(h);
  return h == 0.0 || (a >= 0x1p-1020 && a <= 0x1p1020);
}
// fmin(q, l) for operands that are not signalling NaNs (q a product, l an arithmetic result
// or a finite load): v_min_f64 itself.  fmin's lowering first quiets l with a v_max_f64
// (l, l) on every row of a sweep, which is pure issue cost there.
__device__ __forceinline__ double fmin_q(double q, double l) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(q), "v"(l));
  return r;
}
// fmax(a, |m|) for operands that are not signalling NaNs (a running max, m a min of a
// product): v_max_f64 with the abs source modifier, one instruction.  fmax(a, fabs(m))
// lowers to a canonicalising v_max_f64 (|m|, |m|) first when m comes from inline asm.
__device__ __forceinline__ double fmax_abs_q(double a, double m) {
  double r;
  asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(m));
  return r;
}
__device__ __forceinline__ double hild_step(double t, double h, double rinv, double l, double &nl) {
  if (hild_rok(h) && isfinite(l)) {
    const double m = fmin(t * rinv, l);
    nl = l - m;
    return -m;
  }
  const double w = __builtin_fma(h, l, -t) / h;
  nl = w > 0 ? w : 0.0;
  return nl - l;
}

// predMat.m with A = diag(a), B = ones, evaluated on the structure of Abar:
// identical nonzero arithmetic to the dense products of orc_predmat.
template <int NP>
__device__ __forceinline__ void predmat_s(const double a[6], const double Cb[7], double (&Phi)[NP][NA],
                                          double (&H)[NP]) {
  double S[6], P[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) { S[j] = 0.0; P[j] = 1.0; }
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) acc = acc + Cb[j] * S[j];
    acc = acc + Cb[6] * 1.0;
    H[k] = acc;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      S[j] = a[j] * S[j] + 1.0;
      P[j] = a[j] * P[j];
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) Phi[k][j] = 0.0 + Cb[j] * P[j];
    double acc2 = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) acc2 = acc2 + Cb[j] * S[j];
    acc2 = acc2 + Cb[6] * 1.0;
    Phi[k][6] = acc2;
  }
}

template <int N>
__device__ __forceinline__ void lu_solve_n(const double Ain[N][N], const double b[N], double x[N]) {
  double A[N][N], y[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    y[i] = b[i];
#pragma unroll
    for (int j = 0; j < N; ++j) A[i][j] = Ain[i][j];
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    // first row of largest |A(i,k)| (strictly greater replaces; NaN never does), with the
    // running maximum in a register: A[p][k] with a run-time p would put A in scratch
    int p = k;
#if MPCEKF_LU_SCRATCH_PIVOT  // the round-3 form, for A/B
#pragma unroll
    for (int i = k + 1; i < N; ++i)
      if (fabs(A[i][k]) > fabs(A[p][k])) p = i;
#else
    double pv = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const double a = fabs(A[i][k]);
      if (a > pv) {
        p = i;
        pv = a;
      }
    }
#endif
    // row swap k <-> p with compile-time indices only
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      if (i == p) {
#pragma unroll
        for (int j = 0; j < N; ++j) { double t = A[k][j]; A[k][j] = A[i][j]; A[i][j] = t; }
        double t = y[k]; y[k] = y[i]; y[i] = t;
      }
    }
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      double l = A[i][k] / A[k][k];
      A[i][k] = l;
#pragma unroll
      for (int j = k + 1; j < N; ++j) A[i][j] = A[i][j] - l * A[k][j];
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int k = 0; k < i; ++k) y[i] = y[i] - A[i][k] * y[k];
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    double t = y[i];
#pragma unroll
    for (int k = i + 1; k < N; ++k) t = t - A[i][k] * x[k];
    x[i] = t / A[i][i];
  }
}

// Cholesky of an SPD N x N (upper R); returns false on a non-positive pivot.
template <int N>
__device__ __forceinline__ bool chol_n(const double E[N][N], double R[N][N]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double s = E[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s = s - R[k][j] * R[k][j];
    if (!(s > 0)) ok = false;
    R[j][j] = sqrt(s);
#pragma unroll
    for (int i = j + 1; i < N; ++i) {
      double t = E[j][i];
#pragma unroll
      for (int k = 0; k < j; ++k) t = t - R[k][j] * R[k][i];
      R[j][i] = t / R[j][j];
    }
  }
  return ok;
}
template <int N>
__device__ __forceinline__ void chol_apply(const double R[N][N], const double b[N], double x[N]) {
  double y[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t = t - R[k][i] * y[k];
    y[i] = t / R[i][i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    double t = y[i];
#pragma unroll
    for (int k = i + 1; k < N; ++k) t = t - R[i][k] * x[k];
    x[i] = t / R[i][i];
  }
}
// MATLAB E\b for symmetric E with positive diagonal: Cholesky, else LU.
template <int N>
__device__ __forceinline__ void mldiv_spd(const double E[N][N], const double R[N][N], bool ok, const double b[N],
                                          double x[N]) {
  if (ok) chol_apply<N>(R, b, x);
  else lu_solve_n<N>(E, b, x);
}

// sigma_min of a symmetric PSD N x N via cyclic Jacobi (orc_sigma_min)
template <int N>
__device__ __forceinline__ double sigma_min_n(const double G[N][N]) {
  double a[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) a[i][j] = G[i][j];
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0, dg = 0.0;
#pragma unroll
    for (int p = 0; p < N; ++p) {
      dg = dg + a[p][p] * a[p][p];
#pragma unroll
      for (int q = p + 1; q < N; ++q) off = off + a[p][q] * a[p][q];
    }
    if (!(off > 1e-36 * dg)) break;
#pragma unroll
    for (int p = 0; p < N - 1; ++p)
#pragma unroll
      for (int q = p + 1; q < N; ++q) {
        double apq = a[p][q];
        if (apq != 0.0) {
          double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
          double t;
          if (fabs(theta) > 1e150) {
            t = 0.5 / theta;
          } else {
            t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
            if (theta < 0) t = -t;
          }
          double c = 1.0 / sqrt(t * t + 1.0), s = t * c, tau = s / (1.0 + c);
          a[p][p] = a[p][p] - t * apq;
          a[q][q] = a[q][q] + t * apq;
          a[p][q] = 0.0;
          a[q][p] = 0.0;
#pragma unroll
          for (int r = 0; r < N; ++r) {
            if (r == p || r == q) continue;
            double g = a[r][p], h = a[r][q];
            double gn = g - s * (h + g * tau), hn = h + s * (g - h * tau);
            a[r][p] = gn; a[p][r] = gn;
            a[r][q] = hn; a[q][r] = hn;
          }
        }
      }
  }
  double m = fabs(a[0][0]);
#pragma unroll
  for (int i = 1; i < N; ++i)
    if (fabs(a[i][i]) < m) m = fabs(a[i][i]);
  return m;
}

// Linearisation record (EKFmatsHandler outputs)
struct Lin {
  double a[6], Csoc[6], Dsoc, Cv[6], Dv, Cphi[6], Dphi, bv, bphi, xhat[6];
};

__device__ __forceinline__ void lin_store(double *o, const Lin &L) {
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    o[0 + k] = L.a[k];
    o[6 + k] = L.Csoc[k];
    o[13 + k] = L.Cv[k];
    o[20 + k] = L.Cphi[k];
    o[29 + k] = L.xhat[k];
  }
  o[12] = L.Dsoc; o[19] = L.Dv; o[26] = L.Dphi; o[27] = L.bv; o[28] = L.bphi;
}
__device__ __forceinline__ void lin_load(const double *o, Lin &L) {
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    L.a[k] = o[0 + k];
    L.Csoc[k] = o[6 + k];
    L.Cv[k] = o[13 + k];
    L.Cphi[k] = o[20 + k];
    L.xhat[k] = o[29 + k];
  }
  L.Dsoc = o[12]; L.Dv = o[19]; L.Dphi = o[26]; L.bv = o[27]; L.bphi = o[28];
}

// The constraint matrix of constraintsMPC.m (all switches on) has a fixed
// pattern: rows [Cu; -Cu; I; -I] are constants and the voltage / eta / SOC rows
// are lower-triangular Toeplitz in the impulse responses Hv, He, Hs.  Only those
// 3*NP numbers are kept; mval() reproduces every entry (with the same signed
// zeros) at compile-time indices.
template <int NP, int NC>
struct ConsT {
  static constexpr int NCON = 4 * NC + 3 * NP;
  double Hv[NP], He[NP], Hs[NP];
  double gam[NCON];
};

template <int NP, int NC>
__device__ __forceinline__ double mval(const ConsT<NP, NC> &C, int i, int k) {
  if (i < NC) return k <= i ? 1.0 : 0.0;                              // Cu
  if (i < 2 * NC) return -((k <= i - NC) ? 1.0 : 0.0);                // -Cu
  if (i < 3 * NC) return (i - 2 * NC) == k ? 1.0 : 0.0;               // I
  if (i < 4 * NC) return -((i - 3 * NC) == k ? 1.0 : 0.0);            // -I
  if (i < 4 * NC + NP) { int r = i - 4 * NC; return k <= r ? C.Hv[r - k] : 0.0; }          // G_v
  if (i < 4 * NC + 2 * NP) { int r = i - 4 * NC - NP; return -(k <= r ? C.He[r - k] : 0.0); }  // -G_e
  int r = i - 4 * NC - 2 * NP;
  return k <= r ? C.Hs[r - k] : 0.0;                                   // G_soc
}

// constraintsMPC.m:11-112 for NP x NC (terminal row off, as runMPC)
template <int NP, int NC>
__device__ __forceinline__ void constraints_s(const KCfg &cf, const Lin &L, const double dx[NA], double uk_1,
                                              double SOCk_1, const double (&Phis)[NP][NA], const double (&Hs)[NP],
                                              ConsT<NP, NC> &C) {
  int nr = 0;
#pragma unroll
  for (int i = 0; i < NC; ++i) C.gam[nr + i] = (cf.u_max - uk_1) * 1.0;
  nr += NC;
#pragma unroll
  for (int i = 0; i < NC; ++i) C.gam[nr + i] = -(cf.u_min - uk_1) * 1.0;
  nr += NC;
#pragma unroll
  for (int i = 0; i < NC; ++i) C.gam[nr + i] = cf.du_max * 1.0;
  nr += NC;
#pragma unroll
  for (int i = 0; i < NC; ++i) C.gam[nr + i] = -cf.du_min * 1.0;
  nr += NC;
  double Phi[NP][NA], Cb[7];
#pragma unroll
  for (int k = 0; k < 6; ++k) Cb[k] = L.Cv[k];
  Cb[6] = L.Dv;
  predmat_s<NP>(L.a, Cb, Phi, C.Hv);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) acc = acc + Phi[i][k] * dx[k];
    double rhs = acc + L.bv * 1.0;
    C.gam[nr + i] = cf.v_max - rhs;
  }
  nr += NP;
#pragma unroll
  for (int k = 0; k < 6; ++k) Cb[k] = L.Cphi[k];
  Cb[6] = L.Dphi;
  predmat_s<NP>(L.a, Cb, Phi, C.He);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) acc = acc + Phi[i][k] * dx[k];
    double rhs = acc + L.bphi * 1.0;
    C.gam[nr + i] = -cf.phise_min + rhs;
  }
  nr += NP;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    C.Hs[i] = Hs[i];
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) acc = acc + Phis[i][k] * dx[k];
    double rhs = acc + SOCk_1 * 1.0;
    C.gam[nr + i] = cf.zmax * 1.0 - rhs;
  }
}

struct MpcOut {
  double uk, J_unc, J_fin;
  int nexec, nviol;
};

// iterMPC.m:50-51,85-86 cost J = ||e - G*DU||^2 + DU'*Ru*DU
template <int NP, int NC>
__device__ __forceinline__ double mpc_cost(const double (&Hs)[NP], const double (&e)[NP], double Ru,
                                           const double (&du)[NC]) {
  double J = 0.0, Jq = 0.0;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + (j <= i ? Hs[i - j] : 0.0) * du[j];
    double rr = e[i] - acc;
    J = J + rr * rr;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) acc = acc + (Ru * (c == k ? 1.0 : 0.0)) * du[k];
    Jq = Jq + acc * du[c];
  }
  return J + Jq;
}

// mpcData.cost.norm_DU = norm(DU,2) (iterMPC.m:92): square root of the sequential sum
template <int NC>
__device__ __forceinline__ double norm_du(const double (&DU)[NC]) {
  double s2 = 0.0;
#pragma unroll
  for (int j = 0; j < NC; ++j) s2 = s2 + DU[j] * DU[j];
  return sqrt(s2);
}

// Per-step mpcData.cost outputs (runMPC.m:63-69 / iterMPC.m:89-95) of a finished iterMPC
__device__ __forceinline__ void cost_out(const KIO &io, int64_t c, double J_fin, int nviol, double ndu) {
  if (io.jfin_out) io.jfin_out[c] = J_fin;
  if (io.nviol_out) io.nviol_out[c] = nviol;
  if (io.normdu_out) io.normdu_out[c] = ndu;
}

template <int NP, int NC>
struct MpcSetupT {
  ConsT<NP, NC> Cn;
  double E[NC][NC], F[NC], e[NP], Ru, DU[NC];
};

// iterMPC.m:17-66: predictions, adaptive Ru, unconstrained LS solve, constraint
// stack and the violation test.  Returns true when hildreth.m must run.
// smin_cache (optional): GsocT*Gsoc and its sigma_min for one Gsoc; when this cell's
// GsocT*Gsoc is bitwise the cached one, the cached sigma_min is the value
// sigma_min_n would return (same inputs, same code), so the Jacobi is skipped.
// iterMPC.m:17-48 up to E: predictions, F, GsocT*Gsoc and its sigma_min, Ru, E
template <int NP, int NC>
__device__ __forceinline__ void mpc_core(const KCfg &cf, const Lin &L, double uk_1, double (&dx)[NA],
                                         double (&Phis)[NP][NA], double (&Hs)[NP], MpcSetupT<NP, NC> &P,
                                         double (&GtG)[NC][NC], const double *smin_cache) {
#pragma unroll
  for (int k = 0; k < 6; ++k) dx[k] = L.xhat[k];
  dx[6] = uk_1;
  double Cb[7];
#pragma unroll
  for (int k = 0; k < 6; ++k) Cb[k] = L.Csoc[k];
  Cb[6] = L.Dsoc;
  predmat_s<NP>(L.a, Cb, Phis, Hs);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < NA; ++k) acc = acc + Phis[i][k] * dx[k];
    P.e[i] = cf.ref * 1.0 - acc;
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) acc = acc + (-2 * (j <= i ? Hs[i - j] : 0.0)) * P.e[i];
    P.F[j] = acc;
  }
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < NP; ++i) acc = acc + (a <= i ? Hs[i - a] : 0.0) * (b <= i ? Hs[i - b] : 0.0);
      GtG[a][b] = acc;
    }
  double smin;
  bool hit = false;
  if (smin_cache) {
    hit = true;
#pragma unroll
    for (int a = 0; a < NC; ++a)
#pragma unroll
      for (int b = 0; b < NC; ++b)
        hit = hit && __double_as_longlong(GtG[a][b]) == __double_as_longlong(smin_cache[a * NC + b]);
  }
  if (hit) smin = smin_cache[NC * NC];
  else smin = sigma_min_n<NC>(GtG);
  double nF = 0.0;
#pragma unroll
  for (int j = 0; j < NC; ++j) nF = nF + P.F[j] * P.F[j];
  nF = sqrt(nF);
  P.Ru = (nF / (2 * cf.du_max * sqrt((double)NC))) - smin;
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) P.E[a][b] = 2 * (GtG[a][b] + P.Ru * (a == b ? 1.0 : 0.0));
}

template <int NP, int NC>
__device__ __forceinline__ bool mpc_setup(const KCfg &cf, const Lin &L, double uk_1, double SOCk_1,
                                          MpcSetupT<NP, NC> &P, MpcOut &o, const double *smin_cache = nullptr) {
  constexpr int NCON = 4 * NC + 3 * NP;
  double dx[NA], Phis[NP][NA], Hs[NP], GtG[NC][NC];
  mpc_core<NP, NC>(cf, L, uk_1, dx, Phis, Hs, P, GtG, smin_cache);
  double mE[NC][NC];
#pragma unroll
  for (int a = 0; a < NC; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b) mE[a][b] = -P.E[a][b];
  lu_solve_n<NC>(mE, P.F, P.DU);
  o.J_unc = mpc_cost<NP, NC>(Hs, P.e, P.Ru, P.DU);
  constraints_s<NP, NC>(cf, L, dx, uk_1, SOCk_1, Phis, Hs, P.Cn);
  int nv = 0;
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + mval(P.Cn, i, j) * P.DU[j];
    if (acc - P.Cn.gam[i] > 0) nv++;
  }
  return nv > 0;
}

// iterMPC.m:75-95 after the (optional) Hildreth solve
template <int NP, int NC>
__device__ __forceinline__ void mpc_finish(const ConsT<NP, NC> &Cn, const double (&e)[NP], double Ru,
                                           const double (&DU)[NC], double &uk_1, MpcOut &o) {
  constexpr int NCON = 4 * NC + 3 * NP;
  double uk = DU[0] + uk_1;
  uk_1 = uk;
  o.uk = uk;
  int nviol = 0;
#pragma unroll
  for (int i = 0; i < NCON; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) acc = acc + mval(Cn, i, j) * DU[j];
    if (acc - Cn.gam[i] > 1e-9) nviol++;
  }
  o.nviol = nviol;
  o.J_fin = mpc_cost<NP, NC>(Cn.Hs, e, Ru, DU);
}

// ---------------------------------------------------------------------------
// iterMPC.m:53-60 stability diagnostics: Kmpc = first row of E\(GsocT*Phisoc),
// CL = Abar - Bbar*Kmpc, mpcData.poles = eig(CL), mpcData.sv = svd(CL)
// ---------------------------------------------------------------------------
// E is mpc_core's (the bits iterMPC solved with); GsocT*Phisoc sums from +0 in
// ascending prediction row; E\ is MATLAB's SPD rule (Cholesky, else LU).
template <int NP, int NC>
__device__ __forceinline__ void mpc_kmpc(const KCfg &cf, const Lin &L, double uk_1, double (&Km)[NA]) {
  MpcSetupT<NP, NC> P;
  double dx[NA], Phis[NP][NA], Hs[NP], GtG[NC][NC];
  mpc_core<NP, NC>(cf, L, uk_1, dx, Phis, Hs, P, GtG, nullptr);
  double R[NC][NC];
  const bool ok = chol_n<NC>(P.E, R);
  for (int c = 0; c < NA; ++c) {
    double b[NC], y[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < NP; ++i) acc = acc + (j <= i ? Hs[i - j] : 0.0) * Phis[i][c];
      b[j] = acc;
    }
    mldiv_spd<NC>(P.E, R, ok, b, y);
    Km[c] = y[0];
  }
}

// CL of predMat.m's augmentation with A = diag(a), B = ones: rows 0-5 [diag(a) 1],
// row 6 [-Kmpc(1:6), 1 - Kmpc(7)]
__host__ __device__ inline void closed_loop(const double a[6], const double Km[NA], double CL[NA * NA]) {
  for (int i = 0; i < NA * NA; ++i) CL[i] = 0.0;
  for (int i = 0; i < 6; ++i) {
    CL[i * NA + i] = a[i];
    CL[i * NA + 6] = 1.0;
  }
  for (int j = 0; j < 6; ++j) CL[6 * NA + j] = 0.0 - Km[j];
  CL[6 * NA + 6] = 1.0 - Km[6];
}

// per cell: lin [n][35] (this step's EKFmatsHandler record), uk1 [n] (uk_1 before the
// step's iterMPC); poles [n][7][2] (re, im), sv [n][7] (either may be null)
template <int NP, int NC>
__global__ void __launch_bounds__(64) k_cl_diag(const KCfg cf, int64_t n, const double *lin, const double *uk1,
                                                double *poles, double *sv) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  Lin L;
  lin_load(lin + c * 35, L);
  double Km[NA], CL[NA * NA];
  mpc_kmpc<NP, NC>(cf, L, uk1[c], Km);
  closed_loop(L.a, Km, CL);
  if (poles) {
    double re[NA], im[NA];
    eig::eigvals(NA, CL, re, im);
    for (int i = 0; i < NA; ++i) {
      poles[(c * NA + i) * 2] = re[i];
      poles[(c * NA + i) * 2 + 1] = im[i];
    }
  }
  if (sv) {
    double s[NA];
    eig::singvals(NA, CL, s);
    for (int i = 0; i < NA; ++i) sv[c * NA + i] = s[i];
  }
}

}  // namespace mk
