// Hardware probe: cycles per DP VALU op as a function of the number of active
// lanes (exec popcount) for a dependent chain and for 4 independent chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int ILP>
__global__ void __launch_bounds__(256) k_chain(int active, int iters, double a, double b, double *out, long long *cyc) {
  const int lane = threadIdx.x & 63;
  long long t0 = clock64();
  double x[ILP];
#pragma unroll
  for (int k = 0; k < ILP; ++k) x[k] = lane + k;
  if (lane < active) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < ILP; ++k) x[k] = x[k] * a + b;
    }
  }
  long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int k = 0; k < ILP; ++k) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

int main() {
  const int nblk = 256, nthr = 256, iters = 2000;
  double *out;
  long long *cyc;
  (void)hipMalloc(&out, nblk * nthr * 8);
  (void)hipMalloc(&cyc, nblk * nthr / 64 * 8);
  std::vector<long long> h(nblk * nthr / 64);
  for (int ilp : {1, 4})
    for (int grid : {1, nblk})
      for (int act : {64, 48, 33, 32, 17, 16, 5, 1}) {
        for (int rep = 0; rep < 2; ++rep) {
          if (ilp == 1) hipLaunchKernelGGL(k_chain<1>, dim3(grid), dim3(nthr), 0, 0, act, iters, 0.999, 1e-3, out, cyc);
          else hipLaunchKernelGGL(k_chain<4>, dim3(grid), dim3(nthr), 0, 0, act, iters, 0.999, 1e-3, out, cyc);
          (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h.data(), cyc, grid * nthr / 64 * 8, hipMemcpyDeviceToHost);
        long long mx = 0, mn = 1LL << 62;
        for (int w = 0; w < grid * nthr / 64; ++w) { mx = std::max(mx, h[w]); mn = std::min(mn, h[w]); }
        double ops = (double)iters * 8 * ilp * 2;  // mul + add per step
        printf("ILP %d grid %3d active %2d: cycles/op min %.2f max %.2f\n", ilp, grid, act, mn / ops, mx / ops);
      }
  return 0;
}
