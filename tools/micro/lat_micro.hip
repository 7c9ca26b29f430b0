// Dependent-issue latency of the FP64 operations on the Hildreth chain, one wave per
// SIMD (what k_hild runs at), and the ds_read_b128 -> use latency.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/lat_micro.hip -o tools/micro/lat_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int N = 1024;

#define CHAIN(NAME, BODY)                                                                        \
  __global__ void NAME(double *out, long long *cyc, double a, double b) {                        \
    double x = a + threadIdx.x * 1e-9, y = b;                                                    \
    long long t0 = clock64();                                                                    \
    _Pragma("unroll 64") for (int i = 0; i < N; ++i) { BODY; }                                   \
    long long t1 = clock64();                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                              \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                             \
  }

CHAIN(k_fma, x = __builtin_fma(x, y, 1e-300))
CHAIN(k_mul, x = x * y)
CHAIN(k_add, x = x + y)
CHAIN(k_max, x = fmax(x, y) * 1.0)
CHAIN(k_fma2, x = __builtin_fma(x, y, 1e-300); y = __builtin_fma(y, x, -1e-300))

__global__ void k_lds(double *out, long long *cyc, double a, double b) {
  __shared__ double2 s[64 * 64];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) s[i] = make_double2(0.0, (double)((i + 1) % 64));
  __syncthreads();
  int idx = l;
  double acc = 0.0;
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    const double2 v = s[(idx & 63) * 64 + l];
    idx = (int)v.y;  // dependent address chain
    acc += v.x;
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc + idx;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char *name, K kern, int blocks, int threads, double per) {
  double *d;
  long long *c;
  hipMalloc(&d, (size_t)blocks * threads * 8);
  hipMalloc(&c, blocks * 8);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, c, 1.0, 0.999999);
  hipDeviceSynchronize();
  std::vector<long long> h(blocks);
  hipMemcpy(h.data(), c, blocks * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-6s blocks %4d x %3d: median %.2f cycles per dependent op\n", name, blocks, threads,
         h[blocks / 2] / per);
  hipFree(d);
  hipFree(c);
}

int main() {
  for (int blocks : {1, 256}) {
    run("fma", k_fma, blocks, 256, N);
    run("mul", k_mul, blocks, 256, N);
    run("add", k_add, blocks, 256, N);
    run("max*1", k_max, blocks, 256, N);
    run("fma2", k_fma2, blocks, 256, 2.0 * N);
    run("lds", k_lds, blocks, 256, N);
  }
  return 0;
}
