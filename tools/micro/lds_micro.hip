// LDS cost of k_hild_wide's access shapes: 16-lane groups reading one address
// (broadcast), lanes reading distinct consecutive doubles, and stores where the 16 lanes
// of a group write one address versus one lane per group (the rest to a private sink).
// Prints clock64 ticks per LDS instruction at 1 / 2 waves per SIMD chip-wide; run under
// rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT for array cycles.
// hipcc -O3 --offload-arch=gfx950 tools/micro/lds_micro.hip -o tools/micro/lds_micro
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int N = 1024;

// MODE 0: read, 16-lane broadcast; 1: read, lane-distinct; 2: store, 16 lanes one address;
// 3: store, lane 0 of a group to the shared slot and the others to distinct slots;
// 4: ds_read_b128 broadcast; 5: lane 0 its group's slot, lanes 1-15 a block-wide zero slot
// (k_hild_wide's K_i read); 6: lanes 0-9 distinct decreasing, 10-15 the zero slot (its M
// entries); 7: k_hild_wide's row mix (5, 0, 6, 4, 2 in turn)
template <int MODE>
__global__ void __launch_bounds__(256) k_lds(double *out, long long *cyc, double a) {
  __shared__ double s[8192];
  const int t = threadIdx.x, g = t >> 4, k = t & 15;
  for (int i = t; i < 8192; i += 256) s[i] = a + i;
  __syncthreads();
  double acc = 0.0;
  const int base = 128 + g * 487;  // k_hild_wide's group stride (CELL_LDS doubles)
  double *p = MODE == 1 ? s + base + k : MODE == 3 && k != 0 ? s + 7800 + (t & 63) : s + base;
  double *pk = k == 0 ? s + base + 300 : s;        // K_i or zero
  double *pm = k < 10 ? s + base + 400 + 9 - k : s;  // M entry or zero
  const double2 *p2 = reinterpret_cast<const double2 *>(s + base);
  long long t0 = clock64();
#pragma unroll 32
  for (int i = 0; i < N; ++i) {
    const int o = i & 63;
    if (MODE == 0 || MODE == 1) {
      acc += p[o];
    } else if (MODE == 2 || MODE == 3) {
      p[o] = acc;
      acc += 1.0;
    } else if (MODE == 4) {
      const double2 h = p2[o];
      acc += h.x * h.y;
    } else if (MODE == 5) {
      acc += pk[o];
    } else if (MODE == 6) {
      acc += pm[o];
    } else {
      const int r = i % 5;
      if (r == 0) acc += pk[o];
      else if (r == 1) acc += p[o + 100];
      else if (r == 2) acc += pm[o];
      else if (r == 3) { const double2 h = p2[o]; acc += h.x * h.y; }
      else p[o + 100] = acc;
    }
  }
  __syncthreads();
  long long t1 = clock64();
  out[blockIdx.x * 256 + t] = acc + s[t];
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char *name, K kern, int blocks) {
  double *d;
  long long *c;
  hipMalloc(&d, (size_t)blocks * 256 * 8);
  hipMalloc(&c, blocks * 8);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, c, 1.0);
  hipDeviceSynchronize();
  std::vector<long long> h(blocks);
  hipMemcpy(h.data(), c, blocks * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-22s %5d blocks: median %.2f ticks per LDS instruction per wave\n", name, blocks, h[blocks / 2] / (double)N);
  hipFree(d);
  hipFree(c);
}

int main() {
  for (int blocks : {256, 512}) {
    run("read broadcast16", k_lds<0>, blocks);
    run("read distinct", k_lds<1>, blocks);
    run("store same-addr16", k_lds<2>, blocks);
    run("store lane0+sink", k_lds<3>, blocks);
    run("read_b128 broadcast16", k_lds<4>, blocks);
    run("read K pattern", k_lds<5>, blocks);
    run("read M pattern", k_lds<6>, blocks);
    run("row mix", k_lds<7>, blocks);
  }
  return 0;
}
