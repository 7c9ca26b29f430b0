// k_cell's corner-record access pattern in isolation: what one lane per cell pays to
// read and write back its 4 corner EKF records ([ncells][NM][REC] fp64, corners m0,
// m0+1, m0+nZ, m0+nZ+1), so FETCH_SIZE / WRITE_SIZE of k_cell can be read against a
// calibrated floor for the same pattern.
//   k_once   : the 4 whole records loaded together (20 x 16-B loads in flight per
//              record), a dependent sum, the 4 records stored.
//   k_split  : xhat (40 B) of the 4 records first, a ~20k-cycle dependent FMA chain
//              (getVariables' place), then Sigma (120 B) of each, stored -- the
//              two-visit pattern of k_cell.
//   k_stream : the same bytes as k_once, but record r of cell c at [r][c] per lane
//              (coalesced 16-B streaming) -- the access-shape-independent floor.
// REC=20 is the library layout (160 B); -DPAD=24 pads the record to 192 B.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/rec_micro.hip -o rec_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#ifndef PAD
#define PAD 20
#endif
constexpr int NX = 5, REC = 20, RS = PAD, NM = 63, NZP = 9, NTP = 7;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ void corners(int64_t c, int m[4]) {
  const uint32_t h = hsh((uint32_t)c * 2654435761u);
  const int iT = h % (NTP - 1), iZ = (h >> 8) % (NZP - 1);
  m[0] = iT * NZP + iZ; m[1] = m[0] + 1; m[2] = m[0] + NZP; m[3] = m[2] + 1;
}

__global__ void __launch_bounds__(256) k_once(int64_t n, double *ekf, double *out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  int m[4];
  corners(c, m);
  double v[4][REC];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double2 *p = reinterpret_cast<const double2 *>(ekf + ((size_t)c * NM + m[j]) * RS);
#pragma unroll
    for (int i = 0; i < REC / 2; ++i) { const double2 t = p[i]; v[j][2 * i] = t.x; v[j][2 * i + 1] = t.y; }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < REC; ++i) s = __builtin_fma(s, 0.5, v[j][i]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double2 *p = reinterpret_cast<double2 *>(ekf + ((size_t)c * NM + m[j]) * RS);
#pragma unroll
    for (int i = 0; i < REC / 2; ++i) p[i] = make_double2(v[j][2 * i] + s * 0.0, v[j][2 * i + 1]);
  }
  out[c] = s;
}

__global__ void __launch_bounds__(256) k_split(int64_t n, double *ekf, double *out, int spin) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  int m[4];
  corners(c, m);
  double x[4][NX];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double *r = ekf + ((size_t)c * NM + m[j]) * RS;
    const double2 *p = reinterpret_cast<const double2 *>(r);
    const double2 a = p[0], b = p[1];
    x[j][0] = a.x; x[j][1] = a.y; x[j][2] = b.x; x[j][3] = b.y; x[j][4] = r[4];
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < NX; ++i) s = __builtin_fma(s, 0.5, x[j][i]);
  for (int k = 0; k < spin; ++k) s = __builtin_fma(s, 0.999999, 1e-9);  // getVariables' place
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    double *r = ekf + ((size_t)c * NM + m[j]) * RS;
    double S[15];
    S[0] = r[NX];
    const double2 *p = reinterpret_cast<const double2 *>(r + NX + 1);
#pragma unroll
    for (int i = 0; i < 7; ++i) { const double2 t = p[i]; S[1 + 2 * i] = t.x; S[2 + 2 * i] = t.y; }
    double t = s;
#pragma unroll
    for (int i = 0; i < 15; ++i) t = __builtin_fma(t, 0.5, S[i]);
    double2 *q = reinterpret_cast<double2 *>(r);
    double v[REC];
#pragma unroll
    for (int i = 0; i < NX; ++i) v[i] = x[j][i] + t * 0.0;
#pragma unroll
    for (int i = 0; i < 15; ++i) v[NX + i] = S[i];
#pragma unroll
    for (int i = 0; i < REC / 2; ++i) q[i] = make_double2(v[2 * i], v[2 * i + 1]);
    s = t;
  }
  out[c] = s;
}

__global__ void __launch_bounds__(256) k_stream(int64_t n, double *ekf, double *out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double2 *p = reinterpret_cast<double2 *>(ekf);
  double s = 0.0;
  double2 v[4][REC / 2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < REC / 2; ++i) v[j][i] = p[((size_t)(j * REC / 2 + i)) * n + c];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < REC / 2; ++i) s = __builtin_fma(s, 0.5, v[j][i].x + v[j][i].y);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < REC / 2; ++i) p[((size_t)(j * REC / 2 + i)) * n + c] = make_double2(v[j][i].x + s * 0.0, v[j][i].y);
  out[c] = s;
}

__global__ void k_fill(size_t len, double *a) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (size_t)gridDim.x * blockDim.x)
    a[i] = 1e-3 * (double)(i % 977);
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int spin = argc > 3 ? atoi(argv[3]) : 2000;
  const size_t len = (size_t)n * NM * RS;
  double *ekf, *out;
  CK(hipMalloc(&ekf, len * sizeof(double)));
  CK(hipMalloc(&out, n * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, len, ekf);
  CK(hipDeviceSynchronize());
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double alg = 4.0 * 2 * REC * 8;  // bytes per cell: 4 records read + written
  for (int kind = 0; kind < 3; ++kind) {
    for (int w = 0; w < 3; ++w) {
      if (kind == 0) hipLaunchKernelGGL(k_once, g, b, 0, 0, n, ekf, out);
      if (kind == 1) hipLaunchKernelGGL(k_split, g, b, 0, 0, n, ekf, out, spin);
      if (kind == 2) hipLaunchKernelGGL(k_stream, g, b, 0, 0, n, ekf, out);
    }
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) {
      if (kind == 0) hipLaunchKernelGGL(k_once, g, b, 0, 0, n, ekf, out);
      if (kind == 1) hipLaunchKernelGGL(k_split, g, b, 0, 0, n, ekf, out, spin);
      if (kind == 2) hipLaunchKernelGGL(k_stream, g, b, 0, 0, n, ekf, out);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    printf("{\"kernel\": \"%s\", \"cells\": %lld, \"rec_stride\": %d, \"us\": %.2f, \"alg_bytes_per_cell\": %.0f, \"alg_GBs\": %.1f}\n",
           kind == 0 ? "k_once" : kind == 1 ? "k_split" : "k_stream", (long long)n, RS, us, alg, alg * n / (us * 1e3));
  }
  CK(hipFree(ekf));
  CK(hipFree(out));
  return 0;
}
