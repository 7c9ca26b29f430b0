// FP64 VALU issue rate of one wave against two and four sharing a SIMD: 8 independent fma
// chains per lane (no dependence stalls), blocks of 256 / 512 / 1024 threads on every CU,
// so 1 / 2 / 4 waves per SIMD.  Prints shader cycles per FP64 instruction per wave and per
// SIMD (what a lone wave's Hildreth row can issue).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/issue_micro.hip -o tools/micro/issue_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int N = 4096;

template <int OP>
__global__ void k_issue(double *out, long long *cyc, double a, double b) {
  double x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = a + (threadIdx.x + k) * 1e-9;
  long long t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (OP == 0) x[k] = __builtin_fma(x[k], b, 1e-300);
      if (OP == 1) x[k] = x[k] * b;
      if (OP == 2) x[k] = x[k] + b;
      if (OP == 3) x[k] = __builtin_fmaf((float)x[k], (float)b, 1e-30f);  // fp32 for reference
    }
  }
  long long t1 = clock64();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
static double run(int block, int grid) {
  double *out;
  long long *cyc;
  const int waves = grid * block / 64;
  hipMalloc(&out, sizeof(double) * grid * block);
  hipMalloc(&cyc, sizeof(long long) * waves);
  hipLaunchKernelGGL(k_issue<OP>, dim3(grid), dim3(block), 0, 0, out, cyc, 1.0, 1.0000001);
  hipDeviceSynchronize();
  std::vector<long long> h(waves);
  hipMemcpy(h.data(), cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
  hipFree(out);
  hipFree(cyc);
  std::sort(h.begin(), h.end());
  return (double)h[waves / 2] / (N * 8.0);  // median cycles per instruction per wave
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const char *names[4] = {"v_fma_f64", "v_mul_f64", "v_add_f64", "v_fma_f32"};
  for (int op = 0; op < 4; ++op) {
    for (int wps : {1, 2, 4}) {
      const int block = 256 * wps;
      double c = op == 0 ? run<0>(block, cus) : op == 1 ? run<1>(block, cus) : op == 2 ? run<2>(block, cus)
                                                                                  : run<3>(block, cus);
      std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr_per_wave\": %.2f, "
                  "\"cycles_per_instr_per_simd\": %.2f}\n",
                  names[op], wps, c, c / wps);
    }
  }
  return 0;
}
