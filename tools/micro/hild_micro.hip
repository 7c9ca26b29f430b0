// Micro-benchmark of the Hildreth sweep (k_hild's inner loop) on captured
// problems (tools/hild_problems.npz -> hild_problems.bin by hild_micro.py).
// Reports cycles per sweep for one wave alone and for a full chip of waves.
#include "../../mpc-ekf4fastcharge_amd/csrc/mpcekf_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <vector>

using namespace mk;

// problem record: Hv[5] He[5] Hs[5] gam[23] E[4] F[2] lam0[23]  = 67 doubles
constexpr int PREC_M = 67;

__global__ void __launch_bounds__(256) k_micro(const double *pr, int nprob, int maxIter, double tol, double *lam_out,
                                                int *nexec, long long *cyc, long long *rt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const double *p = pr + (size_t)(c % nprob) * PREC_M;
  Cons Cn;
  double E[NC][NC], F[NC], K[NCON], L[NCON];
  for (int i = 0; i < NP; ++i) { Cn.Hv[i] = p[i]; Cn.He[i] = p[5 + i]; Cn.Hs[i] = p[10 + i]; }
  for (int i = 0; i < NCON; ++i) { Cn.gam[i] = p[15 + i]; L[i] = p[44 + i]; }
  E[0][0] = p[38]; E[0][1] = p[39]; E[1][0] = p[40]; E[1][1] = p[41];
  F[0] = p[42]; F[1] = p[43];
  {
    double y[NC], R[NC][NC];
    bool ok = chol_n<NC>(E, R);
    mldiv_spd<NC>(E, R, ok, F, y);
    ConsM Mf{Cn};
#pragma unroll
    for (int i = 0; i < NCON; ++i) {
      double sum = 0.0;
#pragma unroll
      for (int k = 0; k < NC; ++k) sum = sum + Mf(i, k) * y[k];
      K[i] = sum + Cn.gam[i];
    }
  }

  long long t0 = clock64(), r0 = wall_clock64();
  extern __shared__ double2 hlds[];
  for (int i = 0; i < NCON; ++i) lam_out[c * NCON + i] = L[i];  // warm start (hild_fast's L0)
  int it;
  (void)hild_fast(Cn, E, L, maxIter, tol, K, false, hild_lane_lds(hlds), lam_out + c * NCON, 1, it);
  long long t1 = clock64(), r1 = wall_clock64();
  for (int i = 0; i < NCON; ++i) lam_out[c * NCON + i] = L[i];
  nexec[c] = it;
  cyc[c] = t1 - t0;
  rt[c] = r1 - r0;
}

// k_hild's solve on the dumped problem records with per-lane cycle counts
__global__ void __launch_bounds__(256) k_probe(const KCfg cf, const KState s, int *it_out, long long *cyc,
                                               long long *rt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= s.n) return;
  it_out[c] = 0;
  cyc[c] = 0;
  rt[c] = 0;
  const bool qp = s.hflag[c] != 0;
  const int64_t n = s.n;
  const double *pb = qp ? s.prob : s.prob;  // passengers reuse their (finite) record; results dropped
  Cons Cn;
  double E[NC][NC], F[NC], K[NCON];
  {
    double y[NC], R[NC][NC];
    for (int a = 0; a < NC; ++a) {
      F[a] = pb[(PB_F + a) * n + c];
      for (int b = 0; b < NC; ++b) E[a][b] = pb[(PB_E + a * NC + b) * n + c];
    }
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
  double lam[NCON];
#pragma unroll
  for (int i = 0; i < NCON; ++i) lam[i] = s.lam[(size_t)i * n + c];

  long long t0 = clock64(), r0 = wall_clock64();
  extern __shared__ double2 hlds[];
  int it;
  (void)hild_fast(Cn, E, lam, cf.max_hild, cf.hild_tol, K, !qp, hild_lane_lds(hlds), s.lam + c, n, it);
  long long t1 = clock64(), r1 = wall_clock64();
  if (!qp) return;
  it_out[c] = it;
  cyc[c] = t1 - t0;
  rt[c] = r1 - r0;
}

struct Replay {
  int64_t n;
  double *dprob, *dlam, *dlam0, *duk1, *duk, *djf;
  int *dhf, *dnv, *dit;
  long long *dcyc, *drt;
  KState st;
};

static bool load_state(const char *path, Replay &R) {
  FILE *f = fopen(path, "rb");
  if (!f) { perror(path); return false; }
  int64_t n;
  if (fread(&n, 8, 1, f) != 1) return false;
  std::vector<double> prob((size_t)PROB_DOUBLES * n), lam((size_t)NCON * n);
  std::vector<int> hflag(n);
  if (fread(prob.data(), 8, prob.size(), f) != prob.size() || fread(lam.data(), 8, lam.size(), f) != lam.size() ||
      fread(hflag.data(), 4, n, f) != (size_t)n) return false;
  fclose(f);
  R.n = n;
  hipMalloc(&R.dprob, prob.size() * 8);
  hipMalloc(&R.dlam, lam.size() * 8);
  hipMalloc(&R.dlam0, lam.size() * 8);
  hipMalloc(&R.duk1, n * 8);
  hipMalloc(&R.duk, n * 8);
  hipMalloc(&R.djf, n * 8);
  hipMalloc(&R.dhf, n * 4);
  hipMalloc(&R.dnv, n * 4);
  hipMalloc(&R.dit, n * 4);
  hipMalloc(&R.dcyc, n * 8);
  hipMalloc(&R.drt, n * 8);
  hipMemcpy(R.dprob, prob.data(), prob.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(R.dlam0, lam.data(), lam.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(R.dhf, hflag.data(), n * 4, hipMemcpyHostToDevice);
  KState st{};
  st.n = n; st.prob = R.dprob; st.lam = R.dlam; st.hflag = R.dhf; st.uk_1 = R.duk1; st.uk = R.duk; st.J_fin = R.djf;
  st.nviol = R.dnv; st.J_unc = R.djf;
  hipMalloc(&st.hslow, sizeof(int));
  hipMemset(st.hslow, 0, sizeof(int));
  R.st = st;
  return true;
}

// interleaved A/B replays of k_hild, then one probe launch each with the in-kernel clock
static int ab_mode(int nfiles, char **files, int reps) {
  std::vector<Replay> R(nfiles);
  for (int i = 0; i < nfiles; ++i) if (!load_state(files[i], R[i])) return 1;
  KCfg cf{};
  cf.max_hild = 100;
  cf.hild_tol = 1e-6;
  KIO io{};
  io.mode = MODE_FUSED;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<std::vector<float>> t(nfiles);
  for (int r = 0; r < reps; ++r)
    for (int i = 0; i < nfiles; ++i) {
      hipMemcpy(R[i].dlam, R[i].dlam0, (size_t)NCON * R[i].n * 8, hipMemcpyDeviceToDevice);
      hipEventRecord(e0);
      launch_hild(cf, R[i].st, io, nullptr);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      t[i].push_back(ms);
    }
  for (int i = 0; i < nfiles; ++i) {
    std::vector<float> v = t[i];
    std::sort(v.begin(), v.end());
    printf("%s: k_hild min %.4f median %.4f max %.4f ms  (all:", files[i], v[0], v[v.size() / 2], v.back());
    for (float x : t[i]) printf(" %.3f", x);
    printf(")\n");
    hipMemcpy(R[i].dlam, R[i].dlam0, (size_t)NCON * R[i].n * 8, hipMemcpyDeviceToDevice);
    hipLaunchKernelGGL(k_probe, dim3((R[i].n + 255) / 256), dim3(256), hild_lds_bytes(), 0, cf, R[i].st, R[i].dit, R[i].dcyc,
                       R[i].drt);
    hipDeviceSynchronize();
    int64_t n = R[i].n;
    std::vector<int> it(n);
    std::vector<long long> cyc(n), rt(n);
    hipMemcpy(it.data(), R[i].dit, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(cyc.data(), R[i].dcyc, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(rt.data(), R[i].drt, n * 8, hipMemcpyDeviceToHost);
    // per wave: max it, cycles, realtime
    std::vector<double> clk, cps;
    for (int64_t w = 0; w < n / 64; ++w) {
      int mi = 0;
      long long mc = 0, mr = 0;
      for (int l = 0; l < 64; ++l) {
        int64_t c = w * 64 + l;
        mi = std::max(mi, it[c]);
        mc = std::max(mc, cyc[c]);
        mr = std::max(mr, rt[c]);
      }
      if (mi >= 100 && mr > 0) { clk.push_back(mc / (mr * 0.01) / 1e3); cps.push_back((double)mc / mi); }
    }
    std::sort(clk.begin(), clk.end());
    std::sort(cps.begin(), cps.end());
    if (!clk.empty())
      printf("   probe: %zu waves at 100 sweeps: clock median %.2f GHz [%.2f..%.2f], clk/sweep median %.0f [%.0f..%.0f]\n",
             clk.size(), clk[clk.size() / 2], clk[0], clk.back(), cps[cps.size() / 2], cps[0], cps.back());
  }
  return 0;
}

static int state_mode(const char *path, const char *out) {
  FILE *f = fopen(path, "rb");
  if (!f) { perror(path); return 1; }
  int64_t n;
  if (fread(&n, 8, 1, f) != 1) return 1;
  std::vector<double> prob((size_t)PROB_DOUBLES * n), lam((size_t)NCON * n);
  std::vector<int> hflag(n);
  if (fread(prob.data(), 8, prob.size(), f) != prob.size() || fread(lam.data(), 8, lam.size(), f) != lam.size() ||
      fread(hflag.data(), 4, n, f) != (size_t)n) { fprintf(stderr, "short read\n"); return 1; }
  fclose(f);
  double *dprob, *dlam, *dlam0, *duk1, *duk, *djf;
  int *dhf, *dnv, *dit;
  long long *dcyc;
  hipMalloc(&dprob, prob.size() * 8);
  hipMalloc(&dlam, lam.size() * 8);
  hipMalloc(&dlam0, lam.size() * 8);
  hipMalloc(&duk1, n * 8);
  hipMalloc(&duk, n * 8);
  hipMalloc(&djf, n * 8);
  hipMalloc(&dhf, n * 4);
  hipMalloc(&dnv, n * 4);
  hipMalloc(&dit, n * 4);
  hipMalloc(&dcyc, n * 8);
  hipMemcpy(dprob, prob.data(), prob.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dlam0, lam.data(), lam.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dhf, hflag.data(), n * 4, hipMemcpyHostToDevice);
  KCfg cf{};
  cf.max_hild = 100;
  cf.hild_tol = 1e-6;
  KState st{};
  st.n = n; st.prob = dprob; st.lam = dlam; st.hflag = dhf; st.uk_1 = duk1; st.uk = duk; st.J_fin = djf;
  hipMalloc(&st.hslow, sizeof(int));
  hipMemset(st.hslow, 0, sizeof(int));
  st.nviol = dnv; st.J_unc = djf;
  KIO io{};
  io.mode = MODE_FUSED;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(dlam, dlam0, lam.size() * 8, hipMemcpyDeviceToDevice);
    hipEventRecord(e0);
    launch_hild(cf, st, io, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_hild replay: %.4f ms\n", ms);
  }
  hipMemcpy(dlam, dlam0, lam.size() * 8, hipMemcpyDeviceToDevice);
  long long *drt;
  hipMalloc(&drt, n * 8);
  hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), hild_lds_bytes(), 0, cf, st, dit, dcyc, drt);
  hipDeviceSynchronize();
  std::vector<int> it(n);
  std::vector<long long> cyc(n);
  hipMemcpy(it.data(), dit, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(cyc.data(), dcyc, n * 8, hipMemcpyDeviceToHost);
  FILE *o = fopen(out, "wb");
  fwrite(it.data(), 4, n, o);
  fwrite(cyc.data(), 8, n, o);
  fclose(o);
  long long mx = 0;
  int64_t arg = 0;
  for (int64_t c = 0; c < n; ++c) if (cyc[c] > mx) { mx = cyc[c]; arg = c; }
  printf("probe: slowest lane %ld: %lld clk, nexec %d -> %.0f clk/sweep\n", (long)arg, mx, it[arg],
         (double)mx / (it[arg] ? it[arg] : 1));
  return 0;
}

int main(int argc, char **argv) {
  hipFuncSetAttribute((const void *)k_micro, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void *)k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (argc > 3 && std::string(argv[1]) == "--state") return state_mode(argv[2], argv[3]);
  if (argc > 3 && std::string(argv[1]) == "--ab") return ab_mode(argc - 3, argv + 3, atoi(argv[2]));
  const char *path = argc > 1 ? argv[1] : "tools/micro/hild_problems.bin";
  FILE *f = fopen(path, "rb");
  if (!f) { perror(path); return 1; }
  std::vector<double> h;
  double d;
  while (fread(&d, 8, 1, f) == 1) h.push_back(d);
  fclose(f);
  int nprob = (int)(h.size() / PREC_M);
  double *dp, *dl;
  int *dn;
  long long *dc, *dr;
  const int maxN = 65536;
  hipMalloc(&dp, h.size() * 8);
  hipMemcpy(dp, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipMalloc(&dl, (size_t)maxN * NCON * 8);
  hipMalloc(&dn, maxN * 4);
  hipMalloc(&dc, maxN * 8);
  hipMalloc(&dr, maxN * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int rtfreq = 0;
  hipDeviceGetAttribute(&rtfreq, hipDeviceAttributeWallClockRate, 0);  // kHz
  for (int pid = 0; pid < nprob; ++pid) {
    for (int N : {64, 65536}) {
      // same problem in every lane: no divergence, the wave's own sweep latency
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_micro, dim3((N + 255) / 256), dim3(N < 256 ? N : 256), hild_lds_bytes(), 0, dp + pid * PREC_M, 1, 100,
                           1e-6, dl, dn, dc, dr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      int ne;
      long long cy, rt;
      hipMemcpy(&ne, dn, 4, hipMemcpyDeviceToHost);
      hipMemcpy(&cy, dc, 8, hipMemcpyDeviceToHost);
      hipMemcpy(&rt, dr, 8, hipMemcpyDeviceToHost);
      double us = rt / (rtfreq * 1e-3);
      printf("problem %d  lanes %6d  nexec %3d  kernel %.4f ms  wave0: %lld clk  %.2f us  -> %.0f clk/sweep %.3f us/sweep\n",
             pid, N, ne, ms, cy, us, (double)cy / ne, us / ne);
    }
  }
  std::vector<double> lam(NCON);
  hipMemcpy(lam.data(), dl, NCON * 8, hipMemcpyDeviceToHost);
  printf("lam(last problem, lane 0):");
  for (double v : lam) printf(" %.6g", v);
  printf("\n");
  return 0;
}
