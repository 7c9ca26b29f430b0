// mpcekf_io.hip -- small data-movement kernels of the C-ABI (not reference functions):
// selected columns of a cell-major record array gathered into / scattered from a compact
// [n][k] buffer, so a host reads or writes k doubles per cell in one contiguous copy
// (mpcekf_lin_fields: the 14 of EKFmatsHandler's 35 that runMPC.m:95-96 reads).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mpcekf_kernels.hpp"

namespace mk {
int launch_rows(const double *src, int64_t n, const int *rows, int k, double *dst, void *stream);
}

namespace mk {

// dst[c][j] = src[c * stride + slots[j]] (gather) or src[...] = dst[c][j] (scatter), a thread
// per element, consecutive threads on consecutive (c, j): the compact side is coalesced
template <bool SCATTER>
__global__ void __launch_bounds__(256) k_cols(double *rec, int64_t n, int stride, const int *slots, int k,
                                              double *compact) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * k) return;
  const int64_t c = e / k;
  const int j = (int)(e - c * k);
  double *p = rec + c * stride + slots[j];
  if (SCATTER) *p = compact[e];
  else compact[e] = *p;
}

int launch_cols(double *rec, int64_t n, int stride, const int *slots, int k, double *compact, bool scatter,
                void *stream) {
  if (n <= 0 || k <= 0) return 0;
  const int64_t tot = n * k;
  const dim3 g((unsigned)((tot + 255) / 256)), b(256);
  if (scatter) hipLaunchKernelGGL(k_cols<true>, g, b, 0, (hipStream_t)stream, rec, n, stride, slots, k, compact);
  else hipLaunchKernelGGL(k_cols<false>, g, b, 0, (hipStream_t)stream, rec, n, stride, slots, k, compact);
  return (int)hipGetLastError();
}

// dst[c][j] = src[rows[j] * n + c]: rows of a field-major [k][n] block (the per-cell scalar
// state) as a cell-major [n][k] array, so mpcekf_get_scalars' host copy needs no transpose
// on the host (and its _async form none at the synchronisation)
__global__ void __launch_bounds__(256) k_rows(const double *src, int64_t n, const int *rows, int k, double *dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * k) return;
  const int64_t c = e / k;
  const int j = (int)(e - c * k);
  dst[e] = src[(int64_t)rows[j] * n + c];
}

int launch_rows(const double *src, int64_t n, const int *rows, int k, double *dst, void *stream) {
  if (n <= 0 || k <= 0) return 0;
  const int64_t tot = n * k;
  hipLaunchKernelGGL(k_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, src, n, rows, k,
                     dst);
  return (int)hipGetLastError();
}

}  // namespace mk
