// Checks that the division sequence with the divisor-only part (rcp + 2 Newton
// steps) hoisted is bit-identical to the compiler's correctly rounded x / y for
// operands with |x|, |y| in [2^-400, 2^400] (or x == 0): the range where
// v_div_scale / v_div_fmas / v_div_fixup leave the values unchanged.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double rnd(uint64_t h, int emax) {
  // random sign/mantissa, exponent uniform in [-emax, emax]
  const int e = (int)(h % (2 * emax + 1)) - emax;
  const uint64_t bits = ((uint64_t)(e + 1023) << 52) | (mix(h) & 0xFFFFFFFFFFFFFull) | ((h >> 63) << 63);
  return __longlong_as_double((long long)bits);
}

__global__ void k_check(uint64_t seed, long long iters, unsigned long long *bad, unsigned long long *cnt) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long nb = 0, nc = 0;
  for (long long k = 0; k < iters; ++k) {
    const uint64_t h1 = mix(seed ^ (tid * 0x100000001B3ull) ^ (uint64_t)k * 0xD6E8FEB86659FD93ull);
    const uint64_t h2 = mix(h1);
    double y = rnd(h1, 400), x = rnd(h2, 400);
    if ((h2 & 0xFF) == 0) x = 0.0;
    // near-halfway cases: x a product of y and a short mantissa
    if ((h2 & 0x300) == 0x100) x = y * __longlong_as_double((long long)((1023ull << 52) | (mix(h2) & 0xFFFFFFFull) << 24));
    const double ref = x / y;
    double r = __builtin_amdgcn_rcp(y);
    double e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q0 = x * r;
    const double e2 = __builtin_fma(-y, q0, x);
    const double q = __builtin_fma(e2, r, q0);
    nb += __double_as_longlong(q) != __double_as_longlong(ref) && !(q == 0.0 && ref == 0.0);
    nc++;
  }
  atomicAdd(bad, nb);
  atomicAdd(cnt, nc);
}

int main() {
  unsigned long long *d, h[2];
  (void)hipMalloc(&d, 16);
  (void)hipMemset(d, 0, 16);
  hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, 12345ull, 2000ll, d, d + 1);
  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("checked %llu divisions, mismatches %llu\n", h[1], h[0]);
  return h[0] != 0;
}
