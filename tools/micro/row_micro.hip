// Latency of one wide-Hildreth row (k_hild_wide's dependent chain: row term, 16-lane DPP
// tree, the refined division, max, the v update) and of its pieces, with 1 / 2 / 4 waves
// per SIMD.  hipcc -O3 --offload-arch=gfx950 tools/micro/row_micro.hip -o tools/micro/row_micro
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int N = 512;
#pragma clang fp contract(off)

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double tree16(double a) {
  a = a + dpp64<0xB1>(a);
  a = a + dpp64<0x4E>(a);
  a = a + dpp64<0x141>(a);
  a = a + dpp64<0x140>(a);
  return a;
}

__global__ void k_tree(double *out, long long *cyc, double a, double b) {
  double x = a + threadIdx.x * 1e-9;
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; ++i) x = tree16(x) * b;
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_row(double *out, long long *cyc, double a, double b) {
  double v = a + threadIdx.x * 1e-9, li = 0.5, hx = 2.0 + b, hy = 1.0 / hx, m = b * 0.25, kz = 0.125, xx = 1e-3;
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    const double t = tree16(__builtin_fma(m, v, kz));
    const double num = __builtin_fma(hx, li, -t);
    const double q0 = num * hy;
    const double e2 = __builtin_fma(-hx, q0, num);
    const double wf = __builtin_fma(e2, hy, q0);
    const double nl = wf > 0 ? wf : 0.0;
    const double d = nl - li;
    li = nl;
    v = __builtin_fma(xx, d, v);
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = v + li;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma(double *out, long long *cyc, double a, double b) {
  double x = a + threadIdx.x * 1e-9;
  long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N; ++i) x = __builtin_fma(x, b, 1e-300);
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char *name, K kern, int blocks, int threads) {
  double *d;
  long long *c;
  hipMalloc(&d, (size_t)blocks * threads * 8);
  hipMalloc(&c, blocks * 8);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, c, 1.0, 0.999999);
  hipDeviceSynchronize();
  std::vector<long long> h(blocks);
  hipMemcpy(h.data(), c, blocks * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-5s %5d blocks x %4d threads: median %.1f clock64 ticks per iteration\n", name, blocks, threads,
         h[blocks / 2] / (double)N);
  hipFree(d);
  hipFree(c);
}

int main() {
  // 256 threads = 1 wave per SIMD of one CU; 256 blocks of 256 = 1 wave/SIMD chip-wide; 512 = 2; 1024 = 4
  for (int blocks : {1, 256, 512, 1024}) {
    run("fma", k_fma, blocks, 256);
    run("tree", k_tree, blocks, 256);
    run("row", k_row, blocks, 256);
  }
  return 0;
}
