// mpcekf_host.cpp -- C-ABI (include/mpcekf.h) over the gfx950 kernels.
//
// Owns: ROM validation (initKF.m:66-91, iterEKF.m:692-734, OB_step.m:140-158),
// the output-row permutation and LDS blobs, device state allocation, per-cell
// initialisation (initKF/initMPC/first OB_step), the fused step loop and the
// stage entry points.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpcekf.h"
#include "mpcekf_eig.hpp"
#include "mpcekf_kernels.hpp"

using namespace mk;
namespace mk {
int launch_rows(const double *src, int64_t n, const int *rows, int k, double *dst, void *stream);  // mpcekf_io.hip
}

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(MPCEKF_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

constexpr int NCON_BUILT = 4 * 2 + 3 * 5;  // Np = 5, Nc = 2 compiled into the lane-per-cell kernels
int ncon_of(int Np, int Nc) { return 4 * Nc + 3 * Np; }  // constraintsMPC.m, all switches on

template <class T>
int dalloc(T **p, size_t n) {
  *p = nullptr;
  if (n == 0) return MPCEKF_OK;
  HIPCHK(hipMalloc((void **)p, n * sizeof(T)));
  return MPCEKF_OK;
}

// The output side of the stage calls' host copies (round 6): a pool of worker threads that
// copy device-to-host chunks out of the pinned bounce buffer as their DMA completes.  A call
// enqueues each output as chunks of `chunk` bytes, an event recorded after each chunk's DMA;
// a worker waits for that event and copies the chunk to the caller's array.  So the DMA of
// chunk k + 1 overlaps the copy of chunk k, several threads take the page faults of a
// caller's freshly allocated array at once, and an _async call returns with its copies still
// in flight (finished by the next synchronisation).
struct Copier {
  struct Job {
    hipEvent_t ev;
    const char *src;
    char *dst;
    size_t bytes;
  };
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<Job> q;
  size_t busy = 0;
  bool stop = false;
  hipError_t err = hipSuccess;
  std::vector<std::thread> th;
  int device = 0;
  void start(int n, int dev) {
    device = dev;
    for (int i = 0; i < n; ++i) {
      try {
        th.emplace_back([this]() { run(); });
      } catch (...) {  // no thread: the remaining jobs are copied by drain() itself
        break;
      }
    }
  }
  void run() {
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !q.empty(); });
      if (q.empty()) return;  // stop
      Job j = q.front();
      q.pop_front();
      ++busy;
      lk.unlock();
      do_job(j);
      lk.lock();
      --busy;
      if (q.empty() && !busy) idle.notify_all();
    }
  }
  void do_job(const Job &j) {
    hipError_t e = hipEventSynchronize(j.ev);
    if (e == hipSuccess) std::memcpy(j.dst, j.src, j.bytes);
    else {
      std::lock_guard<std::mutex> g(mu);
      if (err == hipSuccess) err = e;
    }
  }
  void push(const Job &j) {
    if (th.empty()) {  // no worker: copied at the synchronisation, in order
      std::lock_guard<std::mutex> g(mu);
      q.push_back(j);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(j);
    }
    cv.notify_one();
  }
  // every queued copy done; returns (and clears) the first HIP error a worker met
  hipError_t drain() {
    std::unique_lock<std::mutex> lk(mu);
    if (th.empty()) {
      while (!q.empty()) {
        Job j = q.front();
        q.pop_front();
        lk.unlock();
        do_job(j);
        lk.lock();
      }
    } else {
      idle.wait(lk, [&] { return q.empty() && !busy; });
    }
    hipError_t e = err;
    err = hipSuccess;
    return e;
  }
  ~Copier() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (std::thread &t : th) t.join();
  }
};

// MPCEKF_COPY_THREADS, else the CPUs this process may use, 1..16 (the workers sleep on their
// events; at 65,536 cells 16 beat 8 by 15 % on the drop-in route, profiles/r06b_*)
int copy_threads() {
  if (const char *e = std::getenv("MPCEKF_COPY_THREADS")) return std::max(0, std::min(64, std::atoi(e)));
  cpu_set_t set;
  int n = 8;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  return std::max(1, std::min(16, n));
}

}  // namespace

struct mpcekf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t n = 0;
  int NM = 0, nz = 0, nzp = 0, ncon = 0;
  bool initialized = false;
  KRom r{};
  KCfg k{};
  KState s{};
  mpcekf_config cfg{};
  // device buffers owned by the context
  double *d_cell_blob = nullptr, *d_plant_blob = nullptr, *d_bulk = nullptr, *d_poly = nullptr;
  double *d_const = nullptr;  // 8 per-cell constant arrays
  double *d_mb = nullptr;     // model-blend EKF state [n][MBREC] (method MB)
  bool mb = false;
  double *d_scal = nullptr;   // 8 scalar state arrays + J_unc, J_fin
  int *d_int = nullptr;       // warn, status, nviol, hflag
  double *d_prob = nullptr;   // k_cell -> k_hild problem records
  double *d_zk = nullptr, *d_zbk = nullptr;
  double *d_bnd = nullptr;    // k_cell -> k_bounds records [NBND][n]
  int *d_xm = nullptr;        // fused step: Xind hand-off iterEKF kernel -> EKFmatsHandler kernel
  double *d_xg = nullptr;
  bool split_cell = false;    // fused step: k_cell as two kernels (MPCEKF_SPLIT_CELL=1; slower, 0.125 vs 0.118 ms)
  bool quad = false;          // fused step: iterEKF in k_ekf4 (lane quad per cell), then k_cell<P_MPC>
  int ekf4_block = 256;       // k_ekf4 launch bound (MPCEKF_EKF4_BLOCK=512 / 1024: 256 / 128 VGPRs)
  int *d_ts = nullptr;        // deferred time update: ts_ekf, ts_plant [n][NM]
  double *d_hist = nullptr;   // input rings hist_p, hist_u [LAZY_H][n]
  long long *d_stamps = nullptr;  // profiling builds: k_cell section stamps
  // wide horizons (Np = 20, Nc = 10; mpcekf_wide.hip): k_cell hands the linearisation over
  bool wide = false;
  KWide w{};
  double *d_lin = nullptr, *d_zsoc = nullptr;  // [n][35], [n]
  double *d_uk1p = nullptr;                      // [n] uk_1 before the step (poles / sv)
  int flush_period = LAZY_H;      // steps between all-model flushes (<= LAZY_H)
  // rolling flush (MPCEKF_FLUSH_ROLL=1, off by default): step t flushes the cell slice
  // t % flush_period on fstream, forked after k_cell and joined before the next step's k_plant.
  // Measured slower (0.287 vs 0.257 ms per step at 65,536 cells, profiles/r03m_roll_ab.txt):
  // every kernel of the step slows by 5-10 us once the step crosses streams.
  bool flush_roll = false;
  hipStream_t fstream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // batches of ncells <= MPCEKF_BOUNDS_SIDE (default 0: off): k_bounds on fstream beside
  // Hildreth.  Both read only what k_cell wrote and neither writes what the other reads.
  // On by default up to 16,384 cells in rounds 4-5 (+1-3 %); with round 6's shorter k_hild the
  // cross-stream fork and join cost more than the overlap at every size (256-16,384 cells,
  // profiles/r06ab_bounds_side_small.txt), so it is an option.
  bool bounds_side = false;
  hipEvent_t ev_bfork = nullptr, ev_bjoin = nullptr;
  // staging for host trajectories / stage IO (grown on demand)
  double *d_tmp = nullptr;
  size_t tmp_bytes = 0;
  // pinned host bounce buffer of the stage entry points' host copies (Xfer), grown on
  // demand; copies above bounce_max bytes (MPCEKF_BOUNCE_MAX, default 256 MiB: every copy of
  // a 65,536-cell stage call is below 15 MiB) go to / from the caller's memory directly
  char *h_bounce = nullptr;
  size_t h_bytes = 0, bounce_max = (size_t)256 << 20;
  // round 6: the buffer is bump-allocated over the calls up to the next synchronisation
  // (xoff), so _async calls keep their regions until their copies finish; outputs leave it
  // in chunks of xchunk bytes (MPCEKF_CHUNK, default 4 MiB), one event each (xev, reused
  // after the synchronisation), copied out by the worker pool `copier`
  size_t xoff = 0, xchunk = (size_t)4 << 20, xhwm = 0;
  std::vector<hipEvent_t> xev;
  size_t xev_used = 0;
  bool xpending = false;
  Copier *copier = nullptr;
  hipError_t next_event(hipEvent_t *e) {
    if (xev_used == xev.size()) {
      hipEvent_t ne = nullptr;
      hipError_t r = hipEventCreateWithFlags(&ne, hipEventDisableTiming);
      if (r != hipSuccess) return r;
      xev.push_back(ne);
    }
    *e = xev[xev_used++];
    return hipSuccess;
  }
  // the synchronisation every synchronous stage call (and mpcekf_sync) ends with: the
  // stream, then every output copy still queued; the bounce buffer and events free again
  int drain() {
    hipError_t e = hipStreamSynchronize(stream);
    hipError_t c = copier ? copier->drain() : hipSuccess;
    xoff = 0;
    xev_used = 0;
    xpending = false;
    if (e != hipSuccess) return fail(MPCEKF_E_HIP, "hipStreamSynchronize: %s", hipGetErrorString(e));
    if (c != hipSuccess) return fail(MPCEKF_E_HIP, "output copy: %s", hipGetErrorString(c));
    return MPCEKF_OK;
  }
  // per-kernel HIP-event timing (mpcekf_set_timing)
  bool timing = false;
  int timing_every = 1;  // sample every timing_every-th step (1 = every step)
  std::vector<hipEvent_t> ev;
  double t_ms[MPCEKF_NKERNELS] = {};
  int64_t t_n[MPCEKF_NKERNELS] = {};
  // soc(z,T) ends and the table temperatures, for SOC0n/p at init (OB_step.m:63-65)
  std::vector<double> tabT, soc_end[2][2];

  // mpcekf_set_graph: fused calls captured into hipGraphs, keyed by the call shape
  bool graph = false;
  struct GraphEntry {
    std::vector<uintptr_t> key;
    hipGraphExec_t exec;
  };
  std::vector<GraphEntry> graphs;
  template <class Fn>
  int graph_launch(const std::vector<uintptr_t> &key, Fn &&launch) {
    for (const GraphEntry &g : graphs)
      if (g.key == key) {
        HIPCHK(hipGraphLaunch(g.exec, stream));
        return MPCEKF_OK;
      }
    HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    const int rc = launch();
    hipGraph_t gr = nullptr;
    hipError_t e = hipStreamEndCapture(stream, &gr);
    if (rc) {
      if (gr) (void)hipGraphDestroy(gr);
      return rc;
    }
    if (e != hipSuccess) return fail(MPCEKF_E_HIP, "graph capture: %s", hipGetErrorString(e));
    hipGraphExec_t ex = nullptr;
    e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (e != hipSuccess) return fail(MPCEKF_E_HIP, "graph instantiate: %s", hipGetErrorString(e));
    if (graphs.size() >= 16) {  // a small cache: oldest shape out
      (void)hipGraphExecDestroy(graphs.front().exec);
      graphs.erase(graphs.begin());
    }
    graphs.push_back({key, ex});
    HIPCHK(hipGraphLaunch(ex, stream));
    return MPCEKF_OK;
  }
  // the stage route's device-resident hand-offs (runMPC.m:88-103 as the drop-ins call it):
  // the last mpcekf_ekf_step's zk and Xind, the last mpcekf_linearize's records, so the next
  // stage call can take NULL for them instead of a host round trip (valid until a fused step,
  // set_state or init_cells; stage_zk / stage_lin say which are current)
  double *d_szk = nullptr, *d_sxg = nullptr, *d_slin = nullptr, *d_sv = nullptr;
  int *d_sxm = nullptr, *d_zslot = nullptr;  // d_zslot: zk(end)'s slot, nz + 1 (mpc_step's NULL soc_k1)
  bool stage_zk = false, stage_lin = false, stage_v = false;
  int stage_bufs() {
    const size_t nzz = (size_t)nz + 2;
    if (!d_sv) HIPCHK(hipMalloc((void **)&d_sv, (size_t)n * sizeof(double)));
    if (!d_zslot) {
      const int zs = nz + 1;
      HIPCHK(hipMalloc((void **)&d_zslot, sizeof(int)));
      HIPCHK(hipMemcpy(d_zslot, &zs, sizeof(int), hipMemcpyHostToDevice));
    }
    if (!d_szk) HIPCHK(hipMalloc((void **)&d_szk, (size_t)n * nzz * sizeof(double)));
    if (!d_sxg) HIPCHK(hipMalloc((void **)&d_sxg, (size_t)n * 4 * sizeof(double)));
    if (!d_sxm) HIPCHK(hipMalloc((void **)&d_sxm, (size_t)n * 4 * sizeof(int)));
    if (!d_slin) HIPCHK(hipMalloc((void **)&d_slin, (size_t)n * MPCEKF_LIN_SIZE * sizeof(double)));
    return MPCEKF_OK;
  }
  int diag_bufs() {  // the linearisation records and uk_1 copy of the poles / sv diagnostics
    if (!d_lin) HIPCHK(hipMalloc((void **)&d_lin, (size_t)n * MPCEKF_LIN_SIZE * sizeof(double)));
    if (!d_uk1p) HIPCHK(hipMalloc((void **)&d_uk1p, (size_t)n * sizeof(double)));
    return MPCEKF_OK;
  }
  // room for `bytes` more of the current epoch's copies: when the buffer is too small, the
  // pending calls are completed first (drain) and the buffer regrown.  A failed pinned
  // allocation is not an error: the buffer stays empty and every copy goes direct (Xfer::fits).
  int bounce(size_t bytes) {
    if (xoff + bytes <= h_bytes) return MPCEKF_OK;
    // grown to the largest epoch seen (a step's _async calls together), so a steady
    // sequence of calls between synchronisations never drains early
    const size_t want = std::max(xoff + bytes, xhwm);
    xhwm = want;
    if (xpending || xoff) {
      int rc = drain();
      if (rc) return rc;
    }
    bytes = want;
    if (bytes <= h_bytes) return MPCEKF_OK;
    if (h_bounce) (void)hipHostFree(h_bounce);
    h_bounce = nullptr;
    h_bytes = 0;
    if (hipHostMalloc((void **)&h_bounce, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      h_bounce = nullptr;
      return MPCEKF_OK;
    }
    h_bytes = bytes;
    return MPCEKF_OK;
  }
  int tmp(size_t bytes) {
    if (bytes <= tmp_bytes) return MPCEKF_OK;
    if (d_tmp) (void)hipFree(d_tmp);
    d_tmp = nullptr;
    tmp_bytes = 0;
    HIPCHK(hipMalloc((void **)&d_tmp, bytes));
    tmp_bytes = bytes;
    return MPCEKF_OK;
  }
};

extern "C" {

int mpcekf_abi_version(void) { return MPCEKF_ABI_VERSION; }

#ifndef MPCEKF_SRC_HASH
#define MPCEKF_SRC_HASH "unknown"
#endif
const char *mpcekf_build_id(void) { return MPCEKF_SRC_HASH; }

const char *mpcekf_last_error(void) { return g_err.c_str(); }

void mpcekf_config_defaults(mpcekf_config *c) {
  std::memset(c, 0, sizeof(*c));
  c->Np = 5;                  // runMPC.m:28
  c->Nc = 2;                  // runMPC.m:29
  c->target_soc = 95;         // runMPC.m:30
  c->Crate = 2;               // runMPC.m:36
  c->u_max = 2;               // runMPC.m:37
  c->du_min = -50;            // runMPC.m:38
  c->du_max = 50;             // runMPC.m:39
  c->v_min = 3.4;             // runMPC.m:40 (not enforced by constraintsMPC.m)
  c->v_max = 4.1;             // runMPC.m:41
  c->phise_min = 0.08;        // runMPC.m:42
  c->z_max = 95.0 / 100;      // runMPC.m:43
  c->z_tol = 0 * 5.0 / 100;   // runMPC.m:44
  c->use_current = c->use_voltage = c->use_eta = 1;  // runMPC.m:33
  c->max_hild = 100;          // initMPC.m:47
  c->hild_tol = 1e-6;         // hildreth.m:39
  c->SigmaV = 1e-3;           // runMPC.m:19
  c->SigmaW = 1e2;            // runMPC.m:18
  for (int i = 0; i < 5; ++i) c->SigmaX0[i] = 1;
  c->SigmaX0[5] = 2e6;        // runMPC.m:17
  c->max_warn = 10;           // iterEKF.m:55
  c->flags = 0;
  c->method = MPCEKF_METHOD_OB;  // runMPC.m:16 blend = 'OutB'
}

// ---------------------------------------------------------------------------
// ROM validation and packing
// ---------------------------------------------------------------------------
static int build_rom(mpcekf_ctx *X, const mpcekf_rom *R) {
  if (!R || !R->T_degC || !R->SOC_pct || !R->A || !R->C || !R->D || !R->tf_code || !R->tf_xloc)
    return fail(MPCEKF_E_ARG, "rom: null array");
  if (R->n != NX) return fail(MPCEKF_E_UNSUPPORTED, "rom: n = %d transient states, kernels are built for 5", R->n);
  if (R->nT < 1 || R->nT > MAXT || R->nZ < 1 || R->nZ > MAXZ)
    return fail(MPCEKF_E_UNSUPPORTED, "rom: grid %dx%d exceeds %dx%d", R->nT, R->nZ, MAXT, MAXZ);
  if (R->nz < NROLE || R->nz > MAXROWS) return fail(MPCEKF_E_UNSUPPORTED, "rom: nz = %d outside [11, 64]", R->nz);
  if (R->tab_ntheta < 2 || R->tab_ntemp < 1 || R->tab_ntemp > MAXTT || !R->tab_T_K)
    return fail(MPCEKF_E_UNSUPPORTED, "rom: electrode tables need ntheta >= 2 and 1 <= ntemp <= %d", MAXTT);
  for (int j = 0; j < R->tab_ntemp; ++j)
    if (!std::isfinite(R->tab_T_K[j]) || (j && !(R->tab_T_K[j] > R->tab_T_K[j - 1])))
      return fail(MPCEKF_E_ROM, "rom: electrode table temperatures must be finite and ascending");
  for (const mpcekf_electrode *e : {&R->neg, &R->pos})
    if (!e->soc0 || !e->soc100 || !e->Uocp || !e->dUocp || !e->k0 || !e->Rf || !e->Cdleff || !e->Uocp1)
      return fail(MPCEKF_E_ROM, "rom: electrode table missing");
  // ABI v3: theta polynomials (both electrodes, every function) and Arrhenius energies
  if (R->tab_npoly != 0 && R->tab_npoly != 4 && R->tab_npoly != KPOLY)
    return fail(MPCEKF_E_ARG, "rom: tab_npoly = %d (0: linear tables, 4: cubic, 6: quintic)", R->tab_npoly);
  for (const mpcekf_electrode *e : {&R->neg, &R->pos}) {
    const double *ps[6] = {e->Uocp_p, e->dUocp_p, e->k0_p, e->Rf_p, e->Cdleff_p, e->Uocp1_p};
    for (int f = 0; f < 6; ++f) {
      const int m = e->nnode[f];
      if (m != 0 && (!R->tab_npoly || m < 2 || !e->node[f] || !e->node_p[f]))
        return fail(MPCEKF_E_ROM, "rom: nnode[%d] = %d needs tab_npoly, >= 2 nodes and their tables", f, m);
      if (R->tab_npoly && m == 0 && !ps[f])
        return fail(MPCEKF_E_ROM, "rom: tab_npoly = %d but polynomial table %d is missing", R->tab_npoly, f);
      for (int j = 0; j < m; ++j)  // strictly ascending, finite; interior nodes inside (0, 1)
        if (!std::isfinite(e->node[f][j]) || (j && !(e->node[f][j] > e->node[f][j - 1])) ||
            (j > 0 && j < m - 1 && !(e->node[f][j] > 0.0 && e->node[f][j] < 1.0)))
          return fail(MPCEKF_E_ROM, "rom: theta nodes of table %d must be finite, ascending, interior in (0, 1)", f);
    }
    for (int f = 0; f < 5; ++f)
      if (!std::isfinite(e->Ea[f])) return fail(MPCEKF_E_ROM, "rom: Ea[%d] is not finite", f);
  }
  for (int i = 1; i < R->nT; ++i)
    if (!(R->T_degC[i] > R->T_degC[i - 1])) return fail(MPCEKF_E_ROM, "rom: T set-points not ascending");
  for (int i = 1; i < R->nZ; ++i)
    if (!(R->SOC_pct[i] > R->SOC_pct[i - 1])) return fail(MPCEKF_E_ROM, "rom: SOC set-points not ascending");
  const int nT = R->nT, nZ = R->nZ, NM = nT * nZ, nz = R->nz, n1 = NX + 1;
  for (int m = 0; m < NM; ++m)
    if (R->A[(size_t)m * n1 + NX] != 1.0) return fail(MPCEKF_E_ROM, "A for model %d has no integrator state (initKF.m:74)", m);
  for (int q = 0; q < nz; ++q)
    if (R->tf_code[q] < 0 || R->tf_code[q] >= MPCEKF_TF_COUNT) return fail(MPCEKF_E_ROM, "rom: bad tf code at row %d", q);

  // --- index resolution (iterEKF.m:610-735) ---
  auto rows_of = [&](int code) {
    std::vector<int> v;
    for (int q = 0; q < nz; ++q)
      if (R->tf_code[q] == code) v.push_back(q);
    return v;
  };
  auto cat = [](std::vector<int> a, const std::vector<int> &b) {
    a.insert(a.end(), b.begin(), b.end());
    return a;
  };
  const double *loc = R->tf_xloc;
  auto at = [&](const std::vector<int> &v, double x) {
    std::vector<int> o;
    for (int q : v)
      if (loc[q] == x) o.push_back(q);
    return o;
  };
  std::vector<int> Ifdl = cat(rows_of(MPCEKF_TF_negIfdl), rows_of(MPCEKF_TF_posIfdl));
  std::vector<int> If = cat(rows_of(MPCEKF_TF_negIf), rows_of(MPCEKF_TF_posIf));
  std::vector<int> Thss = cat(rows_of(MPCEKF_TF_negThetass), rows_of(MPCEKF_TF_posThetass));
  std::vector<int> Phise = cat(rows_of(MPCEKF_TF_negPhise), rows_of(MPCEKF_TF_posPhise));
  std::vector<int> Phie = cat(cat(rows_of(MPCEKF_TF_negPhie), rows_of(MPCEKF_TF_sepPhie)), rows_of(MPCEKF_TF_posPhie));
  std::vector<int> Thetae =
      cat(cat(rows_of(MPCEKF_TF_negThetae), rows_of(MPCEKF_TF_sepThetae)), rows_of(MPCEKF_TF_posThetae));
  struct {
    const char *name;
    std::vector<int> v;
  } singles[] = {{"ifdl at negative-collector", at(Ifdl, 0)}, {"ifdl at positive-collector", at(Ifdl, 3)},
                 {"if at negative-collector", at(If, 0)},     {"if at positive-collector", at(If, 3)},
                 {"thetass at negative-collector", at(Thss, 0)}, {"thetass at positive-collector", at(Thss, 3)},
                 {"phise at negative-collector", at(Phise, 0)}};
  for (auto &s : singles)
    if (s.v.size() != 1) return fail(MPCEKF_E_ROM, "Simulation requires exactly one %s (iterEKF.m:692-725)", s.name);
  const double eps = 2.220446049250313e-16;
  if (Thetae.empty() || loc[Thetae.front()] > 0) return fail(MPCEKF_E_ROM, "Simulation requires thetae at negative-collector!");
  if (loc[Thetae.back()] > 3 + eps || loc[Thetae.back()] < 3 - eps)
    return fail(MPCEKF_E_ROM, "Simulation requires thetae at positive-collector!");
  if (!Phie.empty() && loc[Phie.front()] == 0) Phie.erase(Phie.begin());  // iterEKF.m:728-731
  if (Phie.empty() || loc[Phie.back()] > 3 + eps || loc[Phie.back()] < 3 - eps)
    return fail(MPCEKF_E_ROM, "Simulation requires phie at positive-collector!");
  std::vector<int> negPhise = rows_of(MPCEKF_TF_negPhise);
  if (negPhise.size() < 2) return fail(MPCEKF_E_ROM, "EKFmatsHandler.m:97 needs ind.negPhise(2)");
  // OB_step's own lookups (OB_step.m:131-137) must agree
  auto negat = [&](int code, double x) { return at(rows_of(code), x); };
  if (negat(MPCEKF_TF_negIfdl, 0) != singles[0].v || negat(MPCEKF_TF_posIfdl, 3) != singles[1].v ||
      negat(MPCEKF_TF_negIf, 0) != singles[2].v || negat(MPCEKF_TF_posIf, 3) != singles[3].v ||
      negat(MPCEKF_TF_negThetass, 0) != singles[4].v || negat(MPCEKF_TF_posThetass, 3) != singles[5].v)
    return fail(MPCEKF_E_ROM, "OB_step and iterEKF resolve collector rows differently");
  int role[NROLE];
  role[R_IFDL0] = singles[0].v[0];
  role[R_IFDL3] = singles[1].v[0];
  role[R_IF0] = singles[2].v[0];
  role[R_IF3] = singles[3].v[0];
  role[R_TH0] = singles[4].v[0];
  role[R_TH3] = singles[5].v[0];
  role[R_TE1] = Thetae.front();
  role[R_TEE] = Thetae.back();
  role[R_PHIE] = Phie.back();
  role[R_PHISE0] = singles[6].v[0];
  role[R_NPHISE2] = negPhise[1];
  for (int a = 0; a < NROLE; ++a)
    for (int b = a + 1; b < NROLE; ++b)
      if (role[a] == role[b]) return fail(MPCEKF_E_UNSUPPORTED, "rom: role rows %d and %d coincide", a, b);
  std::vector<int> perm(role, role + NROLE);
  for (int q = 0; q < nz; ++q)
    if (std::find(perm.begin(), perm.end(), q) == perm.end()) perm.push_back(q);
  int nzp = 0;
  for (int cand : {26, 32})
    if (nz <= cand && cell_kernel_supported(cand)) { nzp = cand; break; }
  if (!nzp) return fail(MPCEKF_E_UNSUPPORTED, "rom: nz = %d not built (kernels: 26, 32)", nz);

  unsigned char flags[MAXROWS] = {0}, c0k[MAXROWS] = {0};
  std::vector<unsigned> fl(nz, 0u);
  std::vector<int> c0(nz, C0_ZERO);
  for (int q : rows_of(MPCEKF_TF_negThetass)) fl[q] |= G_NTH;
  for (int q : rows_of(MPCEKF_TF_posThetass)) fl[q] |= G_PTH;
  for (int q : rows_of(MPCEKF_TF_negPhise)) fl[q] |= G_NPHISE;
  for (int q : rows_of(MPCEKF_TF_posPhise)) fl[q] |= G_PPHISE;
  for (int q : Phie) fl[q] |= G_PHIE | (loc[q] == 0 ? G_PHIE0 : 0u);
  for (int q : Thetae) fl[q] |= G_THETAE;
  for (int q : rows_of(MPCEKF_TF_posPhis)) fl[q] |= G_PPHIS;
  for (int q : rows_of(MPCEKF_TF_posPhis)) c0[q] = C0_CHATV0;  // iterEKF.m:553-586 order
  for (int q : rows_of(MPCEKF_TF_negThetass)) c0[q] = C0_RES0N;
  for (int q : rows_of(MPCEKF_TF_posThetass)) c0[q] = C0_RES0P;
  for (int q : rows_of(MPCEKF_TF_negPhise)) c0[q] = C0_DUN;
  for (int q : rows_of(MPCEKF_TF_posPhise)) c0[q] = C0_DUP;
  for (int q : Phie) c0[q] = C0_MDUN;
  KRom &r = X->r;
  std::memset(&r, 0, sizeof(r));
  for (int q = 0; q < nz; ++q) {
    flags[q] = (unsigned char)fl[perm[q]];
    c0k[q] = (unsigned char)c0[perm[q]];
    r.perm[q] = (short)perm[q];
  }
  std::memcpy(r.flags, flags, sizeof flags);
  for (int q = 0; q < nz && q < 32; ++q)  // nz <= nzp <= 32 (checked above)
    for (int b = 0; b < 8; ++b)
      if (flags[q] >> b & 1) r.fmask[b] |= 1u << q;
  std::memcpy(r.c0k, c0k, sizeof c0k);
  r.NM = NM; r.nT = nT; r.nZ = nZ; r.nz = nz; r.nzp = nzp;
  r.nth = R->tab_ntheta; r.nte = R->tab_ntemp;
  r.Ts = R->Ts; r.Q = R->Q; r.F = R->F; r.R = R->R; r.Rc = R->Rc; r.Tref = R->Tref;
  r.th0n = R->neg.theta0; r.th100n = R->neg.theta100; r.th0p = R->pos.theta0; r.th100p = R->pos.theta100;

  // --- electrode tables (mpcekf_kernels.hip ETab): header, then [fn][side][nte][nth] ---
  // (v3: the header without Uocp1, and the rows as polynomials in a global table)
  const int nth = r.nth, nte = r.nte;
  const bool poly = R->tab_npoly != 0;
  const mpcekf_electrode *els[2] = {&R->neg, &R->pos};
  std::vector<double> tabs;
  if (!poly)
    for (const mpcekf_electrode *e : els) tabs.insert(tabs.end(), e->Uocp1, e->Uocp1 + nth);
  for (int j = 0; j < MAXTT; ++j) tabs.push_back(j < nte ? R->tab_T_K[j] : 0.0);
  X->tabT.assign(R->tab_T_K, R->tab_T_K + nte);
  for (int e = 0; e < 2; ++e)
    for (int one = 0; one < 2; ++one) {
      const double *src = one ? els[e]->soc100 : els[e]->soc0;
      X->soc_end[e][one].assign(src, src + nte);
      for (int j = 0; j < MAXTT; ++j) tabs.push_back(j < nte ? src[j] : 0.0);
    }
  // v3 device layout (mpcekf_kernels.hip ETab::f): per function and electrode the nte rows of
  // each theta interval adjacent, [nth-1][nte][KPOLY] (cubics padded with c4 = c5 = 0), or
  // [nth-1][1][KPOLY] when every row is equal (T-invariant: the row blended with itself, the
  // same value); Uocp1 last
  std::vector<double> ptab;
  const int np = R->tab_npoly;
  const size_t nint = (size_t)(nth - 1);
  // the kernels' lookup descriptors (mpcekf_kernels.hip etab_desc): per function and side
  // Ea/R, (off, istride), (jstride, ro), (mapoff, nu) in doubles of ptab; Uocp1 of each side last
  double desc[12][KDESC] = {};
  bool any_nodes = false;
  auto pack2 = [](long long lo, long long hi) {
    const unsigned long long w = (unsigned long long)(uint32_t)lo | (unsigned long long)(uint32_t)hi << 32;
    double d;
    std::memcpy(&d, &w, sizeof d);
    return d;
  };
  auto add_poly = [&](const double *src, int rows) {  // src [rows][nth-1][np] (ABI order)
    for (size_t i = 0; i < nint; ++i)
      for (int j = 0; j < rows; ++j)
        for (int c = 0; c < KPOLY; ++c) ptab.push_back(c < np ? src[((size_t)j * nint + i) * np + c] : 0.0);
  };
  // ABI v4: a function on its own nodes -- its rows [rows][m-1][np] interval-major like v3's,
  // and a bucket map: nu (a power of two) buckets over [0, 1] with at most one interior node
  // inside each, so that floor(theta nu) and one compare give the oracle's segment
  // k = #{j in 1..m-2 : x_j <= theta}; entry u = (k of u / nu, x_k, x_k+1 or +inf, 0)
  auto add_nodes = [&](double *d, const double *x, int m, const double *src, int rows) -> int {
    const int nseg = m - 1;
    int nu = 1;
    for (;; nu *= 2) {
      bool ok = true;
      for (int j = 2; j < m - 1 && ok; ++j)  // interior nodes j-1, j in one bucket?
        ok = std::floor(x[j] * nu) != std::floor(x[j - 1] * nu);
      if (ok) break;
      if (nu >= (1 << 20)) return fail(MPCEKF_E_ROM, "rom: theta nodes closer than 2^-20");
    }
    d[1] = pack2((long long)ptab.size(), (long long)rows * KPOLY);
    d[2] = pack2(rows > 1 ? KPOLY : 0, rows > 1 ? KPOLY : 0);
    for (int i = 0; i < nseg; ++i)
      for (int j = 0; j < rows; ++j)
        for (int c = 0; c < KPOLY; ++c) ptab.push_back(c < np ? src[((size_t)j * nseg + i) * np + c] : 0.0);
    if (ptab.size() & 1) ptab.push_back(0.0);  // 16-byte map entries
    d[3] = pack2((long long)ptab.size(), nu);
    for (int u = 0; u < nu; ++u) {
      const double e = (double)u / nu;  // exact: nu is a power of two
      int k = 0;
      while (k + 1 <= m - 2 && x[k + 1] <= e) ++k;
      ptab.push_back((double)k);
      ptab.push_back(x[k]);
      ptab.push_back(k + 1 <= m - 2 ? x[k + 1] : HUGE_VAL);
      ptab.push_back(0.0);
    }
    any_nodes = true;
    return MPCEKF_OK;
  };
  bool theta_const = true;
  if (const char *ev = std::getenv("MPCEKF_THETA_CONST")) theta_const = std::atoi(ev) != 0;
  for (int fn = 0; fn < 5 && poly; ++fn)  // EF_U, EF_DU, EF_K0, EF_RF, EF_CDL
    for (int sd = 0; sd < 2; ++sd) {
      const mpcekf_electrode *e = els[sd];
      if (e->nnode[fn] >= 2) {  // v4: on its own nodes
        const int m = e->nnode[fn];
        const double *src = e->node_p[fn];
        const size_t rl = (size_t)(m - 1) * np;
        bool same = nte > 1;
        for (int j = 1; j < nte && same; ++j) same = std::memcmp(src, src + j * rl, rl * sizeof(double)) == 0;
        double *d = desc[fn * 2 + sd];
        d[0] = e->Ea[fn] != 0.0 ? e->Ea[fn] / R->R : 0.0;
        int rc = add_nodes(d, e->node[fn], m, src, same ? 1 : nte);
        if (rc) return rc;
        continue;
      }
      const double *src =
          fn == 0 ? e->Uocp_p : fn == 1 ? e->dUocp_p : fn == 2 ? e->k0_p : fn == 3 ? e->Rf_p : e->Cdleff_p;
      bool same = nte > 1;
      for (int j = 1; j < nte && same; ++j)
        same = std::memcmp(src, src + (size_t)j * nint * np, nint * np * sizeof(double)) == 0;
      double *d = desc[fn * 2 + sd];
      const double ea = e->Ea[fn];
      d[0] = ea != 0.0 ? ea / R->R : 0.0;  // oracle: (Ea / R) * (1/Tref - 1/T)
      const int rows = same ? 1 : nte;
      // a theta-invariant function (every interval's coefficients those of interval 0, e.g.
      // a Cdleff or an Arrhenius k0 that depends on T only): istride 0, so every lane reads
      // interval 0's rows -- one broadcast line instead of a 64-lane gather -- and evaluates
      // them at its own s, the same coefficients and the same s as the oracle's interval:
      // the same bits.  MPCEKF_THETA_CONST=0 keeps the gather (A/B).
      bool thc = nint > 1 && theta_const;
      for (int jr = 0; jr < rows && thc; ++jr)
        for (size_t i = 1; i < nint && thc; ++i)
          thc = std::memcmp(src + ((size_t)jr * nint + i) * np, src + (size_t)jr * nint * np, np * sizeof(double)) == 0;
      d[1] = pack2((long long)ptab.size(), thc ? 0 : (long long)rows * KPOLY);  // off, istride
      d[2] = pack2(same ? 0 : KPOLY, (same || nte == 1) ? 0 : KPOLY);          // jstride, ro
      add_poly(src, rows);
    }
  if (!poly)  // v2: [fn][side][nte][nth] in the LDS blob
    for (int fn = 0; fn < 5; ++fn)
      for (const mpcekf_electrode *e : els) {
        const double *t = fn == 0 ? e->Uocp : fn == 1 ? e->dUocp : fn == 2 ? e->k0 : fn == 3 ? e->Rf : e->Cdleff;
        tabs.insert(tabs.end(), t, t + (size_t)nte * nth);
      }
  if (poly)
    for (int sd = 0; sd < 2; ++sd) {
      if (els[sd]->nnode[5] >= 2) {
        int rc = add_nodes(desc[10 + sd], els[sd]->node[5], els[sd]->nnode[5], els[sd]->node_p[5], 1);
        if (rc) return rc;
        continue;
      }
      desc[10 + sd][1] = pack2((long long)ptab.size(), KPOLY);
      add_poly(els[sd]->Uocp1_p, 1);
    }
  if (poly) {
    if (ptab.size() >= (size_t)INT32_MAX) return fail(MPCEKF_E_ROM, "rom: v3 tables exceed 2^31 doubles");
    for (auto &d : desc) tabs.insert(tabs.end(), d, d + KDESC);
  }
  r.npoly = poly ? KPOLY : 0;
  r.nodes = any_nodes ? 1 : 0;
  r.arr = 0;
  for (int f = 0; f < 5; ++f)
    for (int sd = 0; sd < 2; ++sd) r.arr |= poly && els[sd]->Ea[f] != 0.0;
  // k_cell / k_bounds need no Cdleff table, unless k_cell also runs the plant (cell_plant)
  const char *cpe = getenv("MPCEKF_CELL_PLANT");
  bool cell_plant = !(cpe && atoi(cpe) == 0);
  auto cell_tablen_of = [&](bool cp) { return tabs.size() - (cp || poly ? 0 : (size_t)2 * nte * nth); };
  std::vector<double> pts(MAXT + MAXZ, 0.0);
  for (int t = 0; t < nT; ++t) pts[t] = R->T_degC[t] + 273.15;  // ROMmdls(t,z).T (initKF.m:58)
  for (int z = 0; z < nZ; ++z) pts[MAXT + z] = R->SOC_pct[z] / 100;  // ROMmdls(t,z).SOC
  auto Cval = [&](int m, int q, int k) { return R->C[((size_t)m * nz + q) * n1 + k]; };
  auto Dval = [&](int m, int q) { return R->D[(size_t)m * nz + q]; };
  // cell blob: per model [C nzp x 5][D nzp][a 5][a_p a_q, packed Sigma order 15]
  // (+ [res0 of the 9 plant rows] when k_cell runs the plant).  An odd stride in doubles:
  // lanes reading one offset of different models then spread over all LDS banks (an even
  // stride such as 176 folds them onto 2 bank positions).
  int pr[NPK], pc[NPK];
  for (int p = 0, i = 0; p < NX; ++p)
    for (int q = p; q < NX; ++q, ++i) { pr[i] = p; pc[i] = q; }
  std::vector<double> cb;
  auto make_cell_blob = [&](bool cp) {
    r.cell_stride = (nzp * NX + nzp + NX + NPK + (cp ? NPLANT : 0)) | 1;
    cb.assign((size_t)NM * r.cell_stride, 0.0);
    for (int m = 0; m < NM; ++m) {
      double *b = cb.data() + (size_t)m * r.cell_stride;
      for (int q = 0; q < nz; ++q) {
        for (int k = 0; k < NX; ++k) b[q * NX + k] = Cval(m, perm[q], k);  // initKF.m:91 strips res0
        b[nzp * NX + q] = Dval(m, perm[q]);
      }
      for (int k = 0; k < NX; ++k) b[nzp * NX + nzp + k] = R->A[(size_t)m * n1 + k];
      for (int i = 0; i < NPK; ++i)  // Sigma time update coefficients (iterEKF.m:78)
        b[nzp * NX + nzp + NX + i] = R->A[(size_t)m * n1 + pr[i]] * R->A[(size_t)m * n1 + pc[i]];
      if (cp)  // the plant's res0 column (OB_step.m:272-275; Phise rows are not among the 9)
        for (int q = 0; q < NPLANT; ++q) b[nzp * NX + nzp + NX + NPK + q] = Cval(m, perm[q], NX);
    }
    if (cb.size() & 1) cb.push_back(0.0);  // tables at an even offset: 16-byte staging in rom_global mode
    r.cell_tab = (int)cb.size();
    r.cell_tablen = (int)cell_tablen_of(cp);
    cb.insert(cb.end(), tabs.begin(), tabs.begin() + r.cell_tablen);
    cb.insert(cb.end(), pts.begin(), pts.end());
    r.cell_len = (int)cb.size();
    r.cell_plant = cp;
  };
  make_cell_blob(cell_plant);
  // plant blob: per model [C 9 x 5][res0 9][D 9] over role rows 0..8
  std::vector<double> pb((size_t)NM * PREC, 0.0);
  for (int m = 0; m < NM; ++m) {
    double *b = pb.data() + (size_t)m * PREC;
    for (int q = 0; q < NPLANT; ++q) {
      for (int k = 0; k < NX; ++k) b[q * NX + k] = Cval(m, perm[q], k);
      b[NPLANT * NX + q] = Cval(m, perm[q], NX);  // res0 column (Phise rows are not among these)
      b[NPLANT * NX + NPLANT + q] = Dval(m, perm[q]);
    }
    for (int e = 0; e < 6; ++e) b[NPLANT * NX + 2 * NPLANT + e] = R->A[(size_t)m * n1 + e];  // bigA column
  }
  if (pb.size() & 1) pb.push_back(0.0);
  r.plant_tab = (int)pb.size();
  r.plant_tablen = (int)tabs.size();
  pb.insert(pb.end(), tabs.begin(), tabs.end());
  pb.insert(pb.end(), pts.begin(), pts.end());
  r.plant_len = (int)pb.size();
  // bulk tables: the time-update coefficient of every EKF record element (a for xhat,
  // a_p a_q for Sigma) and of every plant state (bigA)
  std::vector<double> bt((size_t)NM * (REC + 6));
  double *cC = bt.data(), *cP = cC + (size_t)NM * REC;
  for (int m = 0; m < NM; ++m) {
    const double *a = R->A + (size_t)m * n1;
    for (int e = 0; e < NX; ++e) cC[m * REC + e] = a[e];
    for (int i = 0; i < NPK; ++i) cC[m * REC + NX + i] = a[pr[i]] * a[pc[i]];
    for (int e = 0; e < 6; ++e) cP[m * 6 + e] = a[e];
  }
  // Model rows and tables staged in LDS when they fit; otherwise (NM above ~75 at the
  // default grid, or MPCEKF_ROM_GLOBAL=1) only the tables are, and the model rows are read
  // from the global blob (L2-resident).  Same arithmetic either way.
  auto lds_need = [&]() { return std::max(std::max(cell_lds_bytes(r), bounds_lds_bytes(r, 1024)), plant_lds_bytes(r)); };
  const char *gev = getenv("MPCEKF_ROM_GLOBAL");
  r.rom_global = gev && atoi(gev) == 1;
  // the plant's extras (res0 column, Cdleff tables) only while the whole cell blob still
  // fits the LDS; otherwise the plain blob and the separate k_plant
  if (cell_plant && !r.rom_global && cell_lds_bytes(r) > 160 * 1024) make_cell_blob(false);
  if (lds_need() > 160 * 1024) r.rom_global = 1;
  if (lds_need() > 160 * 1024)
    return fail(MPCEKF_E_UNSUPPORTED, "rom: %d bytes of electrode tables exceed the 160 KiB LDS", lds_need());
  int rc;
  if (poly) {
    if ((rc = dalloc(&X->d_poly, ptab.size()))) return rc;
    HIPCHK(hipMemcpy(X->d_poly, ptab.data(), ptab.size() * 8, hipMemcpyHostToDevice));
    r.poly = X->d_poly;
  }
  if ((rc = dalloc(&X->d_cell_blob, cb.size()))) return rc;
  if ((rc = dalloc(&X->d_plant_blob, pb.size()))) return rc;
  if ((rc = dalloc(&X->d_bulk, bt.size()))) return rc;
  HIPCHK(hipMemcpy(X->d_cell_blob, cb.data(), cb.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(X->d_plant_blob, pb.data(), pb.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(X->d_bulk, bt.data(), bt.size() * 8, hipMemcpyHostToDevice));
  r.cell_blob = X->d_cell_blob;
  r.plant_blob = X->d_plant_blob;
  r.bulk_tab = X->d_bulk;
  X->NM = NM;
  X->nz = nz;
  X->nzp = nzp;
  return MPCEKF_OK;
}

static int check_cfg(const mpcekf_config *c) {
  if (!(c->Np == 5 && c->Nc == 2) && !wide_supported(c->Np, c->Nc))
    return fail(MPCEKF_E_UNSUPPORTED, "Np=%d Nc=%d: this build compiles the GPU step for Np/Nc = 5/2 and 20/10",
                c->Np, c->Nc);
  if (!c->use_current || !c->use_voltage || !c->use_eta)
    return fail(MPCEKF_E_UNSUPPORTED, "constraint switches must all be on (runMPC.m:33) in this build");
  if (c->max_hild < 1) return fail(MPCEKF_E_ARG, "max_hild < 1");
  if (c->method != MPCEKF_METHOD_OB && c->method != MPCEKF_METHOD_MB)
    return fail(MPCEKF_E_ARG, "method %d: expected MPCEKF_METHOD_OB or _MB (initKF.m:44-49)", c->method);
  return MPCEKF_OK;
}

static void fill_kcfg(const mpcekf_config *c, double Q, KCfg &k) {
  k.SigmaV = c->SigmaV;
  k.SigmaW = c->SigmaW;
  k.ref = c->target_soc;
  k.u_max = c->u_max;
  k.u_min = -Q * c->Crate;  // initMPC.m:66-67
  k.du_min = c->du_min;
  k.du_max = c->du_max;
  k.v_max = c->v_max;
  k.phise_min = c->phise_min;
  k.zmax = c->z_max + c->z_tol;  // constraintsMPC.m:90-91
  k.hild_tol = c->hild_tol;
  k.max_warn = c->max_warn;
  k.max_hild = c->max_hild;
  k.flags = c->flags | (c->method == MPCEKF_METHOD_MB ? KF_MB : 0);
}

int mpcekf_ctx_create(const mpcekf_rom *rom, const mpcekf_config *cfg, int device, int64_t ncells,
                      mpcekf_ctx **out) {
  if (!out || !cfg || ncells < 0) return fail(MPCEKF_E_ARG, "ctx_create: bad argument");
  *out = nullptr;
  int rc = check_cfg(cfg);
  if (rc) return rc;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MPCEKF_E_ARG, "device %d of %d", device, ndev);
  HIPCHK(hipSetDevice(device));
  mpcekf_ctx *X = new (std::nothrow) mpcekf_ctx();
  if (!X) return fail(MPCEKF_E_ARG, "out of host memory");
  X->device = device;
  X->n = ncells;
  X->cfg = *cfg;
  X->ncon = ncon_of(cfg->Np, cfg->Nc);
  X->wide = wide_supported(cfg->Np, cfg->Nc);
  X->mb = cfg->method == MPCEKF_METHOD_MB;
  if ((rc = build_rom(X, rom))) { mpcekf_ctx_destroy(X); return rc; }
  fill_kcfg(cfg, rom->Q, X->k);
  // Diagnostic override (tests/test_gpu_parity.py shows results do not depend on it):
  // MPCEKF_FLUSH_PERIOD in [1, LAZY_H].
  if (const char *e = std::getenv("MPCEKF_FLUSH_PERIOD")) {
    const int v = std::atoi(e);
    if (v >= 1 && v <= LAZY_H) X->flush_period = v;
  }
  // MPCEKF_SPLIT_CELL=1: the fused step's k_cell as two kernels (results identical).
  if (const char *e = std::getenv("MPCEKF_SPLIT_CELL")) X->split_cell = std::atoi(e) != 0;
  // k_ekf4 (a lane quad per cell for iterEKF; needs four distinct corners: nT > 1, nZ > 1).
  // Round 2 measured it against k_cell under 128 / 256-register budgets (512- / 1024-thread
  // blocks): it lost at every batch size (0.080 vs 0.075 ms at 1,024 cells, 0.20 vs 0.11 at
  // 65,536; profiles/r02g_*).  Round 5's small-batch mapping is the 256-thread instantiation
  // (512 registers, no spills) spread one wave per CU, chosen for batches up to
  // MPCEKF_QUAD_MAX cells, default 8,192 (results identical whichever path runs; same-box
  // A/B, profiles/r05e_small_batch.txt: 1,024 cells 0.173 -> 0.160 ms per step, 4,096 0.176
  // -> 0.164, 16,384 0.189 either way).  MPCEKF_QUAD=0/1 forces it.
  const bool quad_ok = rom->nT > 1 && rom->nZ > 1 && cfg->method == MPCEKF_METHOD_OB && !X->wide;
  {
    int64_t quad_max = 8192;
    if (const char *e = std::getenv("MPCEKF_QUAD_MAX")) quad_max = std::atoll(e);
    X->quad = quad_ok && ncells <= quad_max;
  }
  X->ekf4_block = 256;
  if (const char *e = std::getenv("MPCEKF_QUAD")) X->quad = quad_ok && std::atoi(e) != 0;
  if (const char *e = std::getenv("MPCEKF_EKF4_BLOCK")) {
    const int v = std::atoi(e);
    X->ekf4_block = v == 1024 || v == 512 ? v : 256;
  }
  if (const char *e = std::getenv("MPCEKF_GRAPH")) X->graph = std::atoi(e) != 0;  // as mpcekf_set_graph
  // MPCEKF_FLUSH_ROLL=1: the rolling flush schedule (results identical)
  if (const char *e = std::getenv("MPCEKF_FLUSH_ROLL")) X->flush_roll = std::atoi(e) != 0;
  {
    int64_t side_max = 0;
    if (const char *e = std::getenv("MPCEKF_BOUNDS_SIDE")) side_max = std::atoll(e);
    if (const char *e = std::getenv("MPCEKF_BOUNCE_MAX")) X->bounce_max = (size_t)std::atoll(e);
    if (const char *e = std::getenv("MPCEKF_CHUNK")) X->xchunk = std::max<size_t>((size_t)std::atoll(e), 4096);
    X->bounds_side = ncells <= side_max;
  }
  X->copier = new (std::nothrow) Copier();
  if (!X->copier) { mpcekf_ctx_destroy(X); return fail(MPCEKF_E_HIP, "out of host memory"); }
  X->copier->start(copy_threads(), device);
  hipError_t e = hipStreamCreateWithFlags(&X->stream, hipStreamNonBlocking);
  if (e == hipSuccess && (X->flush_roll || X->bounds_side)) {
    e = hipStreamCreateWithFlags(&X->fstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&X->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&X->ev_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&X->ev_bfork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&X->ev_bjoin, hipEventDisableTiming);
  }
  if (e != hipSuccess) { mpcekf_ctx_destroy(X); return fail(MPCEKF_E_HIP, "stream: %s", hipGetErrorString(e)); }
  const size_t n = (size_t)ncells, NM = (size_t)X->NM;
  KState &s = X->s;
  s.n = ncells;
  if ((rc = dalloc(&s.bigx, n * NM * 6)) || (rc = dalloc(&s.ekf, n * NM * REC)) ||
      (rc = dalloc(&X->d_scal, n * 10)) || (rc = dalloc(&s.lam, n * X->ncon)) ||
      (rc = hipMalloc((void **)&X->d_int, (n * 4 + 1) * sizeof(int)) == hipSuccess ? 0 : MPCEKF_E_HIP) || (rc = dalloc(&X->d_prob, n * PROB_DOUBLES)) || (rc = dalloc(&X->d_const, n * 8)) ||
      (rc = dalloc(&X->d_zk, n * (X->nz + 2))) || (rc = dalloc(&X->d_zbk, n * (X->nz + 2))) ||
      (rc = dalloc(&X->d_bnd, n * NBND)) || (rc = dalloc(&X->d_xg, n * 4)) ||
      (rc = hipMalloc((void **)&X->d_xm, n * 4 * sizeof(int)) == hipSuccess ? 0 : MPCEKF_E_HIP) ||
      (rc = dalloc(&X->d_ts, n * NM * 2)) || (rc = dalloc(&X->d_hist, n * LAZY_H * 2)) ||
      (X->mb && (rc = dalloc(&X->d_mb, n * MBREC)))
#ifdef MPCEKF_STAMPS
      || (rc = dalloc(&X->d_stamps, n * NSTAMPS))
#endif
  ) {
    mpcekf_ctx_destroy(X);
    return rc;
  }
  double *sc = X->d_scal;
  s.SOCn = sc; s.SOCp = sc + n; s.x0 = sc + 2 * n; s.S0 = sc + 3 * n; s.priorI = sc + 4 * n;
  s.uk_1 = sc + 5 * n; s.uk = sc + 6 * n; s.vk = sc + 7 * n; s.J_unc = sc + 8 * n; s.J_fin = sc + 9 * n;
  s.warn = X->d_int; s.status = X->d_int + n; s.nviol = X->d_int + 2 * n; s.hflag = X->d_int + 3 * n;
  s.hslow = X->d_int + 4 * n;
  HIPCHK(hipMemset(s.hslow, 0, sizeof(int)));
  s.prob = X->d_prob;
  s.ts_ekf = X->d_ts; s.ts_plant = X->d_ts + n * NM;
  s.hist_p = X->d_hist; s.hist_u = X->d_hist + n * LAZY_H;
  s.mb = X->d_mb;
  s.stamps = X->d_stamps;
  // rows the current launch sequence does not write (k_plant's 12..19 when the plant runs
  // inside k_cell) read back as zero, never as stale allocation contents
  if (X->d_stamps) HIPCHK(hipMemset(X->d_stamps, 0, (size_t)n * NSTAMPS * sizeof(long long)));
  double *cs = X->d_const;
  s.Tc = cs; s.SOC0 = cs + n; s.SOC0n = cs + 2 * n; s.SOC0p = cs + 3 * n;
  if (X->wide) {
    KWide &w = X->w;
    w.Np = cfg->Np; w.Nc = cfg->Nc; w.ncon = X->ncon;
    const size_t nc = (size_t)X->ncon;
    if ((rc = dalloc(&w.prob, n * wide_prob_doubles(w.Np, w.Nc))) || (rc = dalloc(&w.X, nc * n * w.Nc)) ||
        (rc = dalloc(&w.R, (size_t)n * (w.Nc * (w.Nc + 1) / 2))) || (rc = dalloc(&w.K, nc * n)) || (rc = dalloc(&w.hii, nc * n)) || (rc = dalloc(&w.it, n)) ||
        (rc = dalloc(&w.smin, (size_t)w.Nc * w.Nc + 1)) || (rc = dalloc(&X->d_lin, n * MPCEKF_LIN_SIZE)) ||
        (rc = dalloc(&w.q, 1)) || (rc = dalloc(&w.list, n)) || (rc = dalloc(&w.hist, 128)) ||
        (rc = dalloc(&X->d_zsoc, n))) {
      mpcekf_ctx_destroy(X);
      return rc;
    }
    HIPCHK(hipMemset(w.q, 0, sizeof(int)));
    HIPCHK(hipMemset(w.hist, 0, 128 * sizeof(int)));
    HIPCHK(hipMemset(w.it, 0, n * sizeof(int)));  // the first step's sweep prediction
    // mpc_setup's sigma_min cache: GsocT*Gsoc for Csoc = [0 0 0 0 0 -Ts/(3600 Q)] (EKFmatsHandler.m:43-45)
    rc = launch_wide_smin(w, -rom->Ts / (3600 * rom->Q), rom->A, X->stream);
    if (rc) { mpcekf_ctx_destroy(X); return fail(MPCEKF_E_HIP, "smin kernel: %s", hipGetErrorString((hipError_t)rc)); }
    HIPCHK(hipStreamSynchronize(X->stream));
  }
  *out = X;
  return MPCEKF_OK;
}

int mpcekf_ctx_destroy(mpcekf_ctx *X) {
  if (!X) return MPCEKF_OK;
  (void)hipSetDevice(X->device);
  if (X->stream) (void)X->drain();  // pending _async copies finish before their buffers go
  if (X->fstream) (void)hipStreamSynchronize(X->fstream);
  delete X->copier;
  X->copier = nullptr;
  for (hipEvent_t e : X->xev) (void)hipEventDestroy(e);
  for (hipEvent_t e : X->ev) (void)hipEventDestroy(e);
  if (X->ev_fork) (void)hipEventDestroy(X->ev_fork);
  if (X->ev_join) (void)hipEventDestroy(X->ev_join);
  if (X->ev_bfork) (void)hipEventDestroy(X->ev_bfork);
  if (X->ev_bjoin) (void)hipEventDestroy(X->ev_bjoin);
  void *ptrs[] = {X->d_prob, X->d_cell_blob, X->d_plant_blob, X->d_bulk, X->d_const, X->d_scal, X->d_int, X->d_zk,
                  X->d_zbk,       X->d_tmp,        X->s.bigx, X->s.ekf,   X->s.lam,   X->d_ts, X->d_hist, X->d_stamps, X->d_bnd, X->d_xm, X->d_xg,
                  X->w.prob, X->w.X, X->w.R, X->w.K, X->w.hii, X->w.it, X->w.smin, X->d_lin, X->d_zsoc, X->d_mb, X->d_uk1p,
                  X->w.q, X->w.list, X->w.hist, X->d_poly, X->d_szk, X->d_sxg, X->d_sxm, X->d_slin, X->d_sv, X->d_zslot};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  for (auto &g : X->graphs) (void)hipGraphExecDestroy(g.exec);
  if (X->h_bounce) (void)hipHostFree(X->h_bounce);
  if (X->fstream) (void)hipStreamDestroy(X->fstream);
  if (X->stream) (void)hipStreamDestroy(X->stream);
  delete X;
  return MPCEKF_OK;
}

int mpcekf_ctx_config(const mpcekf_ctx *X, mpcekf_config *cfg) {
  if (!X || !cfg) return fail(MPCEKF_E_ARG, "ctx_config: null argument");
  *cfg = X->cfg;
  return MPCEKF_OK;
}

int mpcekf_ctx_info(const mpcekf_ctx *X, int64_t *ncells, int32_t *nmodels, int32_t *nz, int32_t *ncon) {
  if (!X) return fail(MPCEKF_E_ARG, "null ctx");
  if (ncells) *ncells = X->n;
  if (nmodels) *nmodels = X->NM;
  if (nz) *nz = X->nz;
  if (ncon) *ncon = X->ncon;
  return MPCEKF_OK;
}

// soc(z,T) on the host, the sequence of ETab::bracket / ETab::soc (and orc tidx / fsoc)
static double host_soc(const mpcekf_ctx *X, int side, double z, double T) {
  const std::vector<double> &tk = X->tabT;
  const int nte = (int)tk.size();
  const std::vector<double> &a = X->soc_end[side][0], &b = X->soc_end[side][1];
  if (nte == 1) return a[0] + z * (b[0] - a[0]);
  const double Tc = std::fmin(std::fmax(T, tk[0]), tk[nte - 1]);
  int j = 0;
  while (j < nte - 2 && Tc >= tk[j + 1]) ++j;
  const double g = (Tc - tk[j]) / (tk[j + 1] - tk[j]);
  const double s0 = a[j] + g * (a[j + 1] - a[j]), s1 = b[j] + g * (b[j + 1] - b[j]);
  return s0 + z * (s1 - s0);
}

static int check_tc(const double *tc, size_t count) {
  for (size_t i = 0; i < count; ++i)
    if (!(tc[i] <= 100) || !std::isfinite(tc[i]))
      return fail(MPCEKF_E_ARG, "temperature %zu = %g: must be finite and in degC (iterEKF.m:62)", i, tc[i]);
  return MPCEKF_OK;
}

// A stage call's temperature argument (OB_step's Tc, iterEKF's / EKFmatsHandler's Tk)
// becomes the cell's temperature for this and later calls.
static int set_tc(mpcekf_ctx *X, const double *tc, struct Xfer *xf = nullptr);

// initKF.m:30-136, initMPC.m:29-74 and OB_step.m:39-72 for every cell.
int mpcekf_init_cells(mpcekf_ctx *X, const double *soc0_pct, const double *tc_degC) {
  if (X) X->stage_zk = X->stage_lin = X->stage_v = false;  // the stage route's device hand-offs are stale
  if (!X || ((!soc0_pct || !tc_degC) && X->n)) return fail(MPCEKF_E_ARG, "init_cells: null argument");
  HIPCHK(hipSetDevice(X->device));
  const size_t n = (size_t)X->n;
  int rc0 = 0;
  if ((X->n && (rc0 = check_tc(tc_degC, n)))) return rc0;
  std::vector<double> cst(n * 8), sc(n * 10, 0.0);
  for (size_t c = 0; c < n; ++c) {
    double tc = tc_degC[c], soc0 = soc0_pct[c];
    double T = tc + 273.15;  // OB_step.m:63
    double z = soc0 / 100;
    cst[0 * n + c] = tc;
    cst[1 * n + c] = z;                              // ekfData.SOC0 (initKF.m:133)
    cst[2 * n + c] = host_soc(X, 0, z, T);           // SOC0n = soc(SOC0/100, Tk1) (OB_step.m:64)
    cst[3 * n + c] = host_soc(X, 1, z, T);           // SOC0p
    sc[0 * n + c] = cst[2 * n + c];  // SOCnAvg
    sc[1 * n + c] = cst[3 * n + c];  // SOCpAvg
    sc[3 * n + c] = X->cfg.SigmaX0[5];  // ekfData.SigmaX0 (initKF.m:99)
  }
  HIPCHK(hipMemcpyAsync(X->d_const, cst.data(), cst.size() * 8, hipMemcpyHostToDevice, X->stream));
  HIPCHK(hipMemcpyAsync(X->d_scal, sc.data(), sc.size() * 8, hipMemcpyHostToDevice, X->stream));
  HIPCHK(hipMemsetAsync(X->s.lam, 0, n * X->ncon * 8, X->stream));
  HIPCHK(hipMemsetAsync(X->d_int, 0, n * 4 * sizeof(int), X->stream));
  HIPCHK(hipMemsetAsync(X->d_ts, 0, n * X->NM * 2 * sizeof(int), X->stream));  // every model current
  int rc = launch_init_state(X->n, X->NM, X->s.ekf, X->s.bigx, X->cfg.SigmaX0, X->stream);
  if (rc) return fail(MPCEKF_E_HIP, "init kernel: %s", hipGetErrorString((hipError_t)rc));
  if (X->mb) {  // initKF.m:47-48,111-112: xhat = 0, SigmaX = SigmaX0 (6x6)
    std::vector<double> mbs(n * MBREC, 0.0);
    for (size_t c = 0; c < n; ++c)
      for (int p = 0; p <= NX; ++p) mbs[c * MBREC + 6 + p * (NX + 1) + p] = X->cfg.SigmaX0[p];
    HIPCHK(hipMemcpyAsync(X->d_mb, mbs.data(), mbs.size() * 8, hipMemcpyHostToDevice, X->stream));
    HIPCHK(hipStreamSynchronize(X->stream));
  }
  HIPCHK(hipStreamSynchronize(X->stream));
  X->initialized = true;
  return MPCEKF_OK;
}

static int need_init(mpcekf_ctx *X) {
  if (!X) return fail(MPCEKF_E_ARG, "null ctx");
  if (!X->initialized) return fail(MPCEKF_E_STATE, "call mpcekf_init_cells first");
  HIPCHK(hipSetDevice(X->device));
  return MPCEKF_OK;
}

static int lerr(int rc, const char *what) {
  if (rc) return fail(MPCEKF_E_HIP, "%s launch: %s", what, hipGetErrorString((hipError_t)rc));
  return MPCEKF_OK;
}

// runMPC.m:84-111, nsteps times: OB_step -> (all-model advance + EKF time
// update) -> iterEKF measurement update -> EKFmatsHandler -> iterMPC.
int mpcekf_step_ex(mpcekf_ctx *X, int32_t nsteps, const double *tc_degC, const mpcekf_traj *tr,
                   int32_t outputs_on_device) {
  if (X) X->stage_zk = X->stage_lin = X->stage_v = false;  // the stage route's device hand-offs are stale
  int rc = need_init(X);
  if (rc) return rc;
  if (nsteps < 0) return fail(MPCEKF_E_ARG, "nsteps < 0");
  if (tc_degC && !outputs_on_device && (rc = check_tc(tc_degC, (size_t)X->n * (size_t)nsteps))) return rc;
  mpcekf_traj none{};
  if (!tr) tr = &none;
  const bool bounds = X->cfg.flags & MPCEKF_CF_BOUNDS;
  if (tr->zbk && !bounds) return fail(MPCEKF_E_ARG, "step_ex: a boundzk trajectory needs MPCEKF_CF_BOUNDS");
  // boundzk in k_cell itself, or from its hand-off record in k_bounds (the lane-quad
  // k_ekf4 path writes only the record; MB writes boundzk in k_cell)
  const bool bnd_kernel = bounds && !X->mb && (!cell_computes_bounds() || X->quad);
  // OB_step's simStep inside k_cell (KRom::cell_plant): no k_plant launch
  const bool plant_in_cell = X->r.cell_plant && !X->mb;  // k_cell, or k_ekf4's lane quad (quad_plant)
  // hildreth.m at the end of k_cell (Np = 5, one k_cell per step): no k_hild launch
  const bool hild_in_cell = cell_runs_hild() && !X->wide && !X->split_cell && !X->quad;
  const size_t n = (size_t)X->n, per = n * (size_t)nsteps, nzz = (size_t)X->nz + 2;
  // the output fields, their element size and elements per cell-step
  struct F {
    void *host;
    size_t esz, width;
    char *dev;
  } f[] = {{tr->u, 8, 1, nullptr},       {tr->v, 8, 1, nullptr},      {tr->soc, 8, 1, nullptr},
           {tr->phise, 8, 1, nullptr},   {tr->nexec, 4, 1, nullptr},  {tr->x, 8, 6, nullptr},
           {tr->zk, 8, nzz, nullptr},    {tr->zbk, 8, nzz, nullptr},  {tr->J_unc, 8, 1, nullptr},
           {tr->J_fin, 8, 1, nullptr},   {tr->norm_du, 8, 1, nullptr}, {tr->nviol, 4, 1, nullptr},
           {tr->poles, 8, 2 * NA, nullptr}, {tr->sv, 8, NA, nullptr}};
  constexpr int NF = sizeof(f) / sizeof(f[0]);
  const double *dtc = tc_degC;  // [nsteps][n] device copy of the per-step temperatures
  if (outputs_on_device) {
    for (F &e : f) e.dev = (char *)e.host;
  } else {
    size_t need = tc_degC ? ((per * 8 + 255) & ~(size_t)255) : 0;
    for (F &e : f) need += e.host ? ((per * e.width * e.esz + 255) & ~(size_t)255) : 0;
    if ((rc = X->tmp(need + 256))) return rc;
    char *p = (char *)X->d_tmp;
    for (F &e : f)
      if (e.host) { e.dev = p; p += (per * e.width * e.esz + 255) & ~(size_t)255; }
    if (tc_degC) {
      HIPCHK(hipMemcpyAsync(p, tc_degC, per * 8, hipMemcpyHostToDevice, X->stream));
      dtc = (const double *)p;
    }
  }
  auto row = [&](int i, int k) -> char * {  // step k's [ncells][width] block of field i
    return f[i].dev ? f[i].dev + (size_t)k * n * f[i].width * f[i].esz : nullptr;
  };
  // iterMPC.m:53-60 diagnostics: k_cl_diag after the step from its linearisation records
  // and the uk_1 the step's iterMPC used
  const bool diag = f[12].dev || f[13].dev;
  if (diag && (rc = X->diag_bufs())) return rc;
  constexpr int NEV = 8;  // events per step: plant | cell | bounds | hild (+ diag) |, then | flush |, hild start (side)
  if (X->timing && X->ev.size() < (size_t)nsteps * NEV) {
    size_t old = X->ev.size();
    X->ev.resize((size_t)nsteps * NEV);
    for (size_t i = old; i < X->ev.size(); ++i) HIPCHK(hipEventCreate(&X->ev[i]));
  }
  // Deferred all-model time update: step t advances only the models it
  // touches (k_plant: plant corners, k_cell: EKF corners); k_flush brings every model
  // current each LAZY_H steps and at the end of the call, so between calls (stage entry
  // points, get/set_state) every model is current, exactly as after eager updates.
  //
  // Rolling schedule (flush_roll, MPCEKF_FLUSH_ROLL=1): step t < nsteps flushes only the cells of
  // slice t % P (P = flush_period; slice j = [j n / P, (j + 1) n / P)), so each cell is still
  // flushed every P steps and no replay needs more than P <= LAZY_H ring entries.  The slice
  // runs on fstream, forked after k_cell and joined before the next step's k_plant: k_bounds
  // and Hildreth read no timestamp, ring or model record that k_flush writes (k_flush stores
  // only records older than t, and k_bounds reads the corner k_cell updated at t), and
  // k_plant(t + 1) overwrites the ring slot of step t + 1 - LAZY_H only after the join.  The
  // last step flushes every cell on the step's stream (timestamps 0, as before).  Under graph
  // capture the slices stay on the step's stream (same bits, no overlap).
  const bool capturing = X->graph && !X->timing && nsteps > 0;
  const bool roll = X->flush_roll;
  const bool fork = roll && X->fstream && !capturing;
  // k_bounds beside Hildreth (bounds_side); under graph capture it stays on the step's stream
  const bool side = X->bounds_side && bnd_kernel && X->fstream && !capturing;
  const int hstart = side ? 7 : 3;  // the event that opens the Hildreth interval
  const int P = X->flush_period;
  std::vector<char> flushed((size_t)nsteps, 0);
  auto run_steps = [&]() -> int {
    for (int k = 0; k < nsteps; ++k) {
      const int t = k + 1;
      // sampled steps: every timing_every-th (k = every-1, 2 every-1, ...: with every dividing
      // the flush period these include the flush steps) and the last
      const bool sample = X->timing && ((k + 1) % X->timing_every == 0 || k == nsteps - 1);
      hipEvent_t *E = sample ? &X->ev[(size_t)k * NEV] : nullptr;
      if (E) HIPCHK(hipEventRecord(E[0], X->stream));
      if (diag) HIPCHK(hipMemcpyAsync(X->d_uk1p, X->s.uk_1, n * 8, hipMemcpyDeviceToDevice, X->stream));
      if (!plant_in_cell &&
          (rc = lerr(launch_plant(X->r, X->s, X->s.uk, X->s.vk, t, dtc ? dtc + (size_t)k * n : nullptr, X->stream),
                     "plant")))
        return rc;
      if (E) HIPCHK(hipEventRecord(E[1], X->stream));
      KIO io{};
      io.mode = MODE_FUSED;
      io.lazy_t = t;
      io.plant = plant_in_cell;
      io.tc_in = plant_in_cell && dtc ? dtc + (size_t)k * n : nullptr;
      io.hild = hild_in_cell;
      io.stamps = X->d_stamps;
      io.u = (double *)row(0, k);
      io.v = (double *)row(1, k);
      io.soc = (double *)row(2, k);
      io.phise = (double *)row(3, k);
      io.nexec = (int *)row(4, k);
      io.x_out = (double *)row(5, k);
      io.zk = f[6].dev ? (double *)row(6, k) : X->d_zk;
      double *zbk_k = f[7].dev ? (double *)row(7, k) : X->d_zbk;
      io.zbk = bounds ? zbk_k : nullptr;
      io.bnd = bnd_kernel ? X->d_bnd : nullptr;
      io.junc_out = (double *)row(8, k);
      io.jfin_out = (double *)row(9, k);
      io.normdu_out = (double *)row(10, k);
      io.nviol_out = (int *)row(11, k);
      if (diag) io.lin_out = X->d_lin;
      KIO iow{};  // wide horizons: iterMPC in mpcekf_wide.hip from the linearisation record
      if (X->wide) {
        io.lin_out = X->d_lin;
        io.zsoc_out = X->d_zsoc;
        if ((rc = lerr(launch_cell(X->r, X->k, X->s, io, X->stream, P_EKF | P_LIN), "cell"))) return rc;
        iow.mode = MODE_FUSED;
        iow.lin_in = X->d_lin;
        iow.soc_k1_in = X->d_zsoc;
        iow.u = io.u;
        iow.nexec = io.nexec;
        iow.junc_out = io.junc_out;
        iow.jfin_out = io.jfin_out;
        iow.normdu_out = io.normdu_out;
        iow.nviol_out = io.nviol_out;
        if ((rc = lerr(launch_mpc_wide(X->k, X->s, iow, X->w, X->stream), "mpc_wide"))) return rc;
      } else if (X->split_cell || X->quad) {  // iterEKF, then EKFmatsHandler + iterMPC from zk and Xind in HBM
        io.xm_out = X->d_xm;
        io.xg_out = X->d_xg;
        if (X->quad) {
          if ((rc = lerr(launch_ekf4(X->r, X->k, X->s, io, X->stream, X->ekf4_block), "ekf4"))) return rc;
        } else if ((rc = lerr(launch_cell(X->r, X->k, X->s, io, X->stream, P_EKF), "cell"))) {
          return rc;
        }
        KIO io2 = io;
        io2.zk = nullptr;
        io2.zbk = nullptr;
        io2.bnd = nullptr;
        io2.xm_out = nullptr;
        io2.xg_out = nullptr;
        io2.zk_in = io.zk;
        io2.plant = 0;
        io2.tc_in = nullptr;
        io2.xm_in = X->d_xm;
        io2.xg_in = X->d_xg;
        if ((rc = lerr(launch_cell(X->r, X->k, X->s, io2, X->stream, P_MPC), "cell"))) return rc;
      } else if ((rc = lerr(launch_cell(X->r, X->k, X->s, io, X->stream), "cell"))) {
        return rc;
      }
      if (E) HIPCHK(hipEventRecord(E[2], X->stream));
      const bool slice = roll && t < nsteps;
      if (slice) {
        const int j = t % P;
        const int64_t lo = n * j / P, hi = n * (j + 1) / P;
        hipStream_t fs = X->stream;
        if (fork) {
          HIPCHK(hipEventRecord(X->ev_fork, X->stream));
          HIPCHK(hipStreamWaitEvent(X->fstream, X->ev_fork, 0));
          fs = X->fstream;
        }
        if (E) HIPCHK(hipEventRecord(E[5], fs));
        if ((rc = lerr(launch_flush(X->r, X->k, X->s, t, t, fs, lo, hi), "flush"))) return rc;
        if (E) HIPCHK(hipEventRecord(E[6], fs));
        if (fork) HIPCHK(hipEventRecord(X->ev_join, fs));
        flushed[k] = hi > lo;
      }
      // MB: k_cell writes boundzk itself (one 6x6 covariance per cell)
      if (bnd_kernel) {
        hipStream_t bs = X->stream;
        if (side) {
          HIPCHK(hipEventRecord(X->ev_bfork, X->stream));
          HIPCHK(hipStreamWaitEvent(X->fstream, X->ev_bfork, 0));
          bs = X->fstream;
        }
        if ((rc = lerr(launch_bounds(X->r, X->s, X->d_bnd, zbk_k, bs), "bounds"))) return rc;
        if (E && side) HIPCHK(hipEventRecord(E[3], bs));
        if (side) HIPCHK(hipEventRecord(X->ev_bjoin, bs));
      }
      if (E) HIPCHK(hipEventRecord(E[hstart], X->stream));
      if (X->wide) {
        if ((rc = lerr(launch_hild_wide(X->k, X->s, iow, X->w, X->stream), "hild_wide"))) return rc;
      } else if (!hild_in_cell && (rc = lerr(launch_hild(X->k, X->s, io, X->stream), "hild"))) {
        return rc;
      }
      if (diag) {
        double *pk = (double *)row(12, k), *sk = (double *)row(13, k);
        rc = X->wide ? launch_cl_diag_wide(X->k, X->n, X->d_lin, X->d_uk1p, pk, sk, X->stream)
                     : launch_cl_diag(X->k, X->n, X->d_lin, X->d_uk1p, pk, sk, X->stream);
        if ((rc = lerr(rc, "cl_diag"))) return rc;
      }
      if (E) HIPCHK(hipEventRecord(E[4], X->stream));
      // k_bounds done before k_flush or the next step's k_cell rewrites the records it reads
      if (side) HIPCHK(hipStreamWaitEvent(X->stream, X->ev_bjoin, 0));
      if (slice && fork) HIPCHK(hipStreamWaitEvent(X->stream, X->ev_join, 0));
      if (roll ? t == nsteps : (t % P == 0 || t == nsteps)) {
        const bool timed = E && !roll;  // the rolling schedule times its slices only
        if (timed) HIPCHK(hipEventRecord(E[5], X->stream));
        if ((rc = lerr(launch_flush(X->r, X->k, X->s, t, t == nsteps ? 0 : t, X->stream), "flush"))) return rc;
        if (timed) HIPCHK(hipEventRecord(E[6], X->stream));
        flushed[k] = timed;
      }
    }
    return MPCEKF_OK;
  };
  if (capturing) {
    // the call's launches depend only on these (kernel arguments are call-relative:
    // lazy_t = 1..nsteps, the flush schedule, the output rows), so a repeated call shape
    // replays one instantiated graph instead of 5-7 launches per step
    std::vector<uintptr_t> key = {(uintptr_t)nsteps, (uintptr_t)dtc, (uintptr_t)diag, (uintptr_t)bounds};
    for (const F &e : f) key.push_back((uintptr_t)e.dev);
    if ((rc = X->graph_launch(key, run_steps))) return rc;
  } else if ((rc = run_steps())) {
    return rc;
  }
  if (!outputs_on_device)
    for (int i = 0; i < NF; ++i)
      if (f[i].host)
        HIPCHK(hipMemcpyAsync(f[i].host, f[i].dev, per * f[i].width * f[i].esz, hipMemcpyDeviceToHost, X->stream));
  // mpcekf_get_zk returns the last step's zk / boundzk whichever buffers the steps wrote
  if (nsteps > 0 && f[6].dev)
    HIPCHK(hipMemcpyAsync(X->d_zk, row(6, nsteps - 1), n * nzz * 8, hipMemcpyDeviceToDevice, X->stream));
  if (nsteps > 0 && f[7].dev)
    HIPCHK(hipMemcpyAsync(X->d_zbk, row(7, nsteps - 1), n * nzz * 8, hipMemcpyDeviceToDevice, X->stream));
  HIPCHK(hipStreamSynchronize(X->stream));
  if (X->timing) {
    // (start, end) events of plant, cell, bounds, hild, flush
    static const int slot[5] = {MPCEKF_K_PLANT, MPCEKF_K_CELL, MPCEKF_K_BOUNDS, MPCEKF_K_HILD, MPCEKF_K_FLUSH};
    static const int e0[5] = {0, 1, 2, 3, 5};
    for (int k = 0; k < nsteps; ++k)
      for (int j = 0; j < 5; ++j) {
        if ((k + 1) % X->timing_every != 0 && k != nsteps - 1) continue;
        if ((j == 4 && !flushed[k]) || (j == 2 && !bnd_kernel) || (j == 0 && plant_in_cell) ||
            (j == 3 && hild_in_cell && !diag))
          continue;
        float ms = 0;
        const int a = j == 3 ? hstart : e0[j], b = j == 3 ? 4 : e0[j] + 1;
        HIPCHK(hipEventElapsedTime(&ms, X->ev[(size_t)k * NEV + a], X->ev[(size_t)k * NEV + b]));
        X->t_ms[slot[j]] += ms;
        X->t_n[slot[j]] += 1;
      }
  }
  return MPCEKF_OK;
}

int mpcekf_cl_eig(int32_t n, const double *a, double *re, double *im, double *sv) {
  if (n < 1 || n > mk::eig::MAXN || !a) return fail(MPCEKF_E_ARG, "cl_eig: n must be 1..%d", mk::eig::MAXN);
  double r[mk::eig::MAXN], m[mk::eig::MAXN], s[mk::eig::MAXN];
  if (re || im) mk::eig::eigvals(n, a, r, m);
  if (sv) mk::eig::singvals(n, a, s);
  for (int i = 0; i < n; ++i) {
    if (re) re[i] = r[i];
    if (im) im[i] = m[i];
    if (sv) sv[i] = s[i];
  }
  return MPCEKF_OK;
}

int mpcekf_step(mpcekf_ctx *X, int32_t nsteps, const double *tc_degC, double *traj_u, double *traj_v,
                double *traj_soc, double *traj_phise, int32_t *traj_nexec, int32_t outputs_on_device) {
  mpcekf_traj tr{};
  tr.u = traj_u;
  tr.v = traj_v;
  tr.soc = traj_soc;
  tr.phise = traj_phise;
  tr.nexec = traj_nexec;
  return mpcekf_step_ex(X, nsteps, tc_degC, &tr, outputs_on_device);
}

int mpcekf_set_graph(mpcekf_ctx *X, int32_t enable) {
  if (!X) return fail(MPCEKF_E_ARG, "null ctx");
  X->graph = enable != 0;
  return MPCEKF_OK;
}

int mpcekf_set_timing(mpcekf_ctx *X, int32_t enable) {
  if (!X) return fail(MPCEKF_E_ARG, "null ctx");
  X->timing = enable != 0;
  X->timing_every = enable > 1 ? enable : 1;
  return MPCEKF_OK;
}

int mpcekf_get_timing(mpcekf_ctx *X, double *ms_sum, int64_t *launches) {
  if (!X) return fail(MPCEKF_E_ARG, "null ctx");
  for (int j = 0; j < MPCEKF_NKERNELS; ++j) {
    if (ms_sum) ms_sum[j] = X->t_ms[j];
    if (launches) launches[j] = X->t_n[j];
    X->t_ms[j] = 0;
    X->t_n[j] = 0;
  }
  return MPCEKF_OK;
}

// ---- device memory owned by the library ---------------------------------------
// Callers that keep trajectories on the device (bench.py, the GPU tests, a MEX host)
// allocate them here, so a process holds exactly one HIP runtime: the one this
// library links.  A second runtime (e.g. a framework's bundled copy) in the same
// process owns its own HSA queues and address-space bookkeeping; pointers must not
// cross between the two.
int mpcekf_dev_alloc(int device, int64_t bytes, void **ptr) {
  if (!ptr || bytes < 0) return fail(MPCEKF_E_ARG, "dev_alloc: bad argument");
  *ptr = nullptr;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MPCEKF_E_ARG, "dev_alloc: device %d of %d", device, ndev);
  if (bytes == 0) return MPCEKF_OK;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(ptr, (size_t)bytes));
  return MPCEKF_OK;
}

int mpcekf_dev_free(void *ptr) {
  if (ptr) HIPCHK(hipFree(ptr));
  return MPCEKF_OK;
}

static hipMemcpyKind copy_kind(int32_t kind) {
  return kind == MPCEKF_COPY_H2D ? hipMemcpyHostToDevice
       : kind == MPCEKF_COPY_D2H ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
}

int mpcekf_dev_copy(void *dst, const void *src, int64_t bytes, int32_t kind) {
  if (bytes < 0 || kind < MPCEKF_COPY_H2D || kind > MPCEKF_COPY_D2D || (bytes && (!dst || !src)))
    return fail(MPCEKF_E_ARG, "dev_copy: bad argument");
  if (bytes) HIPCHK(hipMemcpy(dst, src, (size_t)bytes, copy_kind(kind)));
  return MPCEKF_OK;
}

int mpcekf_dev_copy2d(void *dst, int64_t dpitch, const void *src, int64_t spitch, int64_t width, int64_t height,
                      int32_t kind) {
  if (width < 0 || height < 0 || dpitch < width || spitch < width || kind < MPCEKF_COPY_H2D ||
      kind > MPCEKF_COPY_D2D || (width && height && (!dst || !src)))
    return fail(MPCEKF_E_ARG, "dev_copy2d: bad argument");
  if (width && height)
    HIPCHK(hipMemcpy2D(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)height, copy_kind(kind)));
  return MPCEKF_OK;
}

int mpcekf_sync(mpcekf_ctx *X) {
  if (!X) return fail(MPCEKF_E_ARG, "null ctx");
  HIPCHK(hipSetDevice(X->device));
  int rc = X->drain();  // the _async stage calls' host outputs are written when this returns
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  return MPCEKF_OK;
}

int mpcekf_get_zk(mpcekf_ctx *X, double *zk, double *boundzk) {
  int rc = need_init(X);
  if (rc) return rc;
  size_t bytes = (size_t)X->n * (X->nz + 2) * 8;
  if (zk) HIPCHK(hipMemcpyAsync(zk, X->d_zk, bytes, hipMemcpyDeviceToHost, X->stream));
  if (boundzk) HIPCHK(hipMemcpyAsync(boundzk, X->d_zbk, bytes, hipMemcpyDeviceToHost, X->stream));
  HIPCHK(hipStreamSynchronize(X->stream));
  return MPCEKF_OK;
}

// ---- stage entry points ----------------------------------------------------
}  // extern "C"
// Host arrays are staged through one device scratch slab.
struct Slab {
  char *base;
  size_t off = 0;
  template <class T>
  T *take(size_t count) {
    T *p = (T *)(base + off);
    off += (count * sizeof(T) + 255) & ~(size_t)255;
    return p;
  }
};
// A stage call's host copies, through the context's pinned bounce buffer: inputs are copied
// into it and sent from there; outputs are DMA'd into it in chunks and copied out by the
// context's worker pool as each chunk's event completes (Copier), which the call's
// synchronisation (finish) waits for -- or, for an _async call (finish_async), the next one.
// Copies straight from / into the caller's pageable arrays let the runtime pin and cache
// those pages; the drop-ins' callers (MATLAB's mxArrays, numpy) free and reallocate their
// arrays every call, and the stage sequence then stalled 10-20 ms in whichever call came
// next (tools/dropin_probe.py: 0.6 ms with every array kept alive, 10-14 ms when freed,
// reused or not allocated; profiles/r05e_dropin_probe.jsonl).
struct Xfer {
  mpcekf_ctx *X;
  // bounced when below the cap and inside the buffer reserved (a copy beyond the
  // reservation goes direct rather than past the buffer's end)
  bool fits(size_t b) const { return b <= X->bounce_max && X->xoff + pad(b) <= X->h_bytes; }
  static size_t pad(size_t b) { return (b + 255) & ~(size_t)255; }
  // capacity for the call's copies: pad(bytes) summed over those that will be bounced
  // (bounce_max caps a copy; MPCEKF_BOUNCE_MAX=0 pins nothing)
  int reserve(const std::vector<size_t> &copies) {
    size_t sum = 0;
    for (size_t b : copies)
      if (b && b <= X->bounce_max) sum += pad(b);
    return sum ? X->bounce(sum) : MPCEKF_OK;
  }
  hipError_t in(void *d, const void *h, size_t b) {
    if (!b) return hipSuccess;
    if (!fits(b)) return hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, X->stream);
    char *p = X->h_bounce + X->xoff;
    X->xoff += pad(b);
    std::memcpy(p, h, b);
    return hipMemcpyAsync(d, p, b, hipMemcpyHostToDevice, X->stream);
  }
  hipError_t out(void *h, const void *d, size_t b) {
    if (!b) return hipSuccess;
    if (!fits(b)) return hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, X->stream);
    char *p = X->h_bounce + X->xoff;
    X->xoff += pad(b);
    for (size_t o = 0; o < b; o += X->xchunk) {
      const size_t len = std::min(X->xchunk, b - o);
      hipError_t e = hipMemcpyAsync(p + o, (const char *)d + o, len, hipMemcpyDeviceToHost, X->stream);
      hipEvent_t ev = nullptr;
      if (e == hipSuccess) e = X->next_event(&ev);
      if (e == hipSuccess) e = hipEventRecord(ev, X->stream);
      if (e != hipSuccess) return e;
      X->copier->push({ev, p + o, (char *)h + o, len});
    }
    return hipSuccess;
  }
  // the synchronous call's end: every output (this call's and any earlier _async call's) written
  int finish() { return X->drain(); }
  // an _async call's end: its copies stay in flight until mpcekf_sync or a synchronous call
  int finish_async() {
    X->xpending = true;
    return MPCEKF_OK;
  }
  int end(bool async) { return async ? finish_async() : finish(); }
};
static int set_tc(mpcekf_ctx *X, const double *tc, Xfer *xf) {
  if (!tc) return MPCEKF_OK;
  int rc = check_tc(tc, (size_t)X->n);
  if (rc) return rc;
  if (xf) HIPCHK(xf->in(X->s.Tc, tc, (size_t)X->n * 8));
  else HIPCHK(hipMemcpyAsync(X->s.Tc, tc, (size_t)X->n * 8, hipMemcpyHostToDevice, X->stream));
  return MPCEKF_OK;
}
extern "C" {

static int plant_step_impl(mpcekf_ctx *X, const double *iapp, const double *tc_degC, double *vcell, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!iapp) return fail(MPCEKF_E_ARG, "plant_step: null argument");
  size_t n = (size_t)X->n;
  Xfer xf{X};
  if ((rc = xf.reserve({n * 8, n * 8, n * 8}))) return rc;
  if ((rc = set_tc(X, tc_degC, &xf))) return rc;
  if ((rc = X->tmp(2 * n * 8 + 512)) || (rc = X->stage_bufs())) return rc;
  Slab sl{(char *)X->d_tmp};
  // Vcell also stays on the device for the next mpcekf_ekf_step (vk = NULL there: runMPC.m:88
  // -> :91 without a host round trip, which an _async plant call needs); vcell may be NULL
  double *di = sl.take<double>(n), *dv = X->d_sv;
  X->stage_v = false;
  HIPCHK(xf.in(di, iapp, n * 8));
  if ((rc = lerr(launch_plant(X->r, X->s, di, dv, 0, nullptr, X->stream), "plant"))) return rc;
  if ((rc = lerr(launch_bulk(X->r, X->k, X->s, di, 1, 0, X->stream), "bulk"))) return rc;
  if (vcell) HIPCHK(xf.out(vcell, dv, n * 8));
  if ((rc = xf.end(async))) return rc;
  X->stage_v = true;
  return MPCEKF_OK;
}
int mpcekf_plant_step(mpcekf_ctx *X, const double *iapp, const double *tc_degC, double *vcell) {
  return plant_step_impl(X, iapp, tc_degC, vcell, false);
}
int mpcekf_plant_step_async(mpcekf_ctx *X, const double *iapp, const double *tc_degC, double *vcell) {
  return plant_step_impl(X, iapp, tc_degC, vcell, true);
}

static int ekf_step_impl(mpcekf_ctx *X, const double *vk, const double *ik, const double *tk_degC, double *zk,
                    double *boundzk, int32_t *xind_model, double *xind_gamma, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!ik) return fail(MPCEKF_E_ARG, "ekf_step: null argument");
  if (!vk && !X->stage_v) return fail(MPCEKF_E_STATE, "ekf_step: NULL vk but no mpcekf_plant_step before it");
  size_t n = (size_t)X->n, nzz = (size_t)X->nz + 2;
  Xfer xf{X};
  if ((rc = xf.reserve({n * 8, n * 8, n * 8, n * nzz * 8, n * nzz * 8, 16 * n, 32 * n})))
    return rc;
  if ((rc = set_tc(X, tk_degC, &xf))) return rc;
  if ((rc = X->tmp((2 * n + n * nzz) * 8 + 2048)) || (rc = X->stage_bufs())) return rc;
  Slab sl{(char *)X->d_tmp};
  double *dvk = sl.take<double>(n), *dik = sl.take<double>(n), *dzb = sl.take<double>(n * nzz);
  // zk and Xind stay on the device for the next mpcekf_linearize (NULL there); each host
  // output is copied only when given
  double *dzk = X->d_szk, *dxg = X->d_sxg;
  int *dxm = X->d_sxm;
  X->stage_zk = X->stage_lin = false;
  if (vk) HIPCHK(xf.in(dvk, vk, n * 8));
  else dvk = X->d_sv;  // the last mpcekf_plant_step's Vcell, on the device
  HIPCHK(xf.in(dik, ik, n * 8));
  // iterEKF.m:55 lock-out must see the state before the time update: the bulk
  // update of a locked-out cell is harmless because the cell is stopped.
  // OB: the all-model time update (iterEKF.m:73-84); MB updates only its blended model (in k_cell)
  if (!X->mb && (rc = lerr(launch_bulk(X->r, X->k, X->s, nullptr, 0, 1, X->stream), "bulk"))) return rc;
  KIO io{};
  io.mode = MODE_EKF;
  io.vk_in = dvk;
  io.ik_in = dik;
  io.zk = dzk;
  io.zbk = boundzk ? dzb : nullptr;
  const bool bnd_kernel = boundzk && !X->mb && !cell_computes_bounds();
  io.bnd = bnd_kernel ? X->d_bnd : nullptr;
  io.xm_out = dxm;
  io.xg_out = dxg;
  if ((rc = lerr(launch_cell(X->r, X->k, X->s, io, X->stream), "cell"))) return rc;
  if (bnd_kernel && (rc = lerr(launch_bounds(X->r, X->s, X->d_bnd, dzb, X->stream), "bounds"))) return rc;
  if (zk) HIPCHK(xf.out(zk, dzk, n * nzz * 8));
  if (boundzk) HIPCHK(xf.out(boundzk, dzb, n * nzz * 8));
  if (xind_model) HIPCHK(xf.out(xind_model, dxm, 4 * n * 4));
  if (xind_gamma) HIPCHK(xf.out(xind_gamma, dxg, 4 * n * 8));
  if ((rc = xf.end(async))) return rc;
  X->stage_zk = true;
  return MPCEKF_OK;
}
int mpcekf_ekf_step(mpcekf_ctx *X, const double *vk, const double *ik, const double *tk_degC, double *zk,
                    double *boundzk, int32_t *xind_model, double *xind_gamma) {
  return ekf_step_impl(X, vk, ik, tk_degC, zk, boundzk, xind_model, xind_gamma, false);
}
int mpcekf_ekf_step_async(mpcekf_ctx *X, const double *vk, const double *ik, const double *tk_degC, double *zk,
                    double *boundzk, int32_t *xind_model, double *xind_gamma) {
  return ekf_step_impl(X, vk, ik, tk_degC, zk, boundzk, xind_model, xind_gamma, true);
}

static int linearize_impl(mpcekf_ctx *X, const double *zk, const int32_t *xind_model, const double *xind_gamma,
                     const double *tk_degC, double *lin, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!zk != !xind_model || !xind_model != !xind_gamma)
    return fail(MPCEKF_E_ARG, "linearize: zk, xind_model and xind_gamma are all given or all NULL");
  if (!zk && !X->stage_zk) return fail(MPCEKF_E_STATE, "linearize: NULL zk / Xind but no mpcekf_ekf_step before it");
  size_t n = (size_t)X->n, nzz = (size_t)X->nz + 2;
  Xfer xf{X};
  if ((rc = xf.reserve({n * 8, n * nzz * 8, 16 * n, 32 * n, n * MPCEKF_LIN_SIZE * 8})))
    return rc;
  if ((rc = set_tc(X, tk_degC, &xf))) return rc;
  if ((rc = X->tmp((n * nzz + 4 * n) * 8 + 4 * n * 4 + 2048)) || (rc = X->stage_bufs())) return rc;
  Slab sl{(char *)X->d_tmp};
  double *dzk = X->d_szk, *dxg = X->d_sxg, *dl = X->d_slin;
  int *dxm = X->d_sxm;
  if (zk) {  // the caller's zk / Xind (a host that changed them after iterEKF)
    dzk = sl.take<double>(n * nzz);
    dxg = sl.take<double>(4 * n);
    dxm = sl.take<int>(4 * n);
    HIPCHK(xf.in(dzk, zk, n * nzz * 8));
    HIPCHK(xf.in(dxm, xind_model, 4 * n * 4));
    HIPCHK(xf.in(dxg, xind_gamma, 4 * n * 8));
  }
  KIO io{};
  io.mode = MODE_LIN;
  io.zk_in = dzk;
  io.xm_in = dxm;
  io.xg_in = dxg;
  io.lin_out = dl;
  X->stage_lin = false;
  if ((rc = lerr(launch_cell(X->r, X->k, X->s, io, X->stream), "cell"))) return rc;
  if (lin) HIPCHK(xf.out(lin, dl, n * MPCEKF_LIN_SIZE * 8));
  if ((rc = xf.end(async))) return rc;
  X->stage_lin = true;
  return MPCEKF_OK;
}
int mpcekf_linearize(mpcekf_ctx *X, const double *zk, const int32_t *xind_model, const double *xind_gamma,
                     const double *tk_degC, double *lin) {
  return linearize_impl(X, zk, xind_model, xind_gamma, tk_degC, lin, false);
}
int mpcekf_linearize_async(mpcekf_ctx *X, const double *zk, const int32_t *xind_model, const double *xind_gamma,
                     const double *tk_degC, double *lin) {
  return linearize_impl(X, zk, xind_model, xind_gamma, tk_degC, lin, true);
}

static int lin_fields_impl(mpcekf_ctx *X, const int32_t *slots, int32_t nslots, const double *set, double *out, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!X->stage_lin) return fail(MPCEKF_E_STATE, "lin_fields: no mpcekf_linearize record on the device");
  if (nslots < 0 || nslots > MPCEKF_LIN_SIZE || (nslots && !slots)) return fail(MPCEKF_E_ARG, "lin_fields: bad slots");
  uint64_t seen = 0;  // a repeated slot would have several threads scatter into one record element
  for (int i = 0; i < nslots; ++i) {
    if (slots[i] < 0 || slots[i] >= MPCEKF_LIN_SIZE) return fail(MPCEKF_E_ARG, "lin_fields: slot %d", slots[i]);
    if (seen >> slots[i] & 1) return fail(MPCEKF_E_ARG, "lin_fields: slot %d given twice", slots[i]);
    seen |= (uint64_t)1 << slots[i];
  }
  if (!nslots || (!set && !out)) return MPCEKF_OK;
  // the slots gathered into / scattered from a compact [ncells][nslots] device buffer, which
  // crosses PCIe in one copy: only the named doubles move (per-slot pitched copies of 8-byte
  // columns cost 3.7 ms for 14 slots at 65,536 cells, profiles/r05b_dropin_capi_65536.json)
  const size_t n = (size_t)X->n, bytes = n * (size_t)nslots * 8;
  if ((rc = X->tmp(bytes + 1024))) return rc;
  Slab sl{(char *)X->d_tmp};
  double *dc = sl.take<double>(n * (size_t)nslots);
  int *ds = sl.take<int>((size_t)nslots);
  Xfer xf{X};
  if ((rc = xf.reserve({(size_t)nslots * sizeof(int), bytes, bytes}))) return rc;
  HIPCHK(xf.in(ds, slots, (size_t)nslots * sizeof(int)));
  if (set) {
    HIPCHK(xf.in(dc, set, bytes));
    if ((rc = lerr(launch_cols(X->d_slin, X->n, MPCEKF_LIN_SIZE, ds, nslots, dc, true, X->stream), "cols"))) return rc;
  }
  if (out) {
    if ((rc = lerr(launch_cols(X->d_slin, X->n, MPCEKF_LIN_SIZE, ds, nslots, dc, false, X->stream), "cols"))) return rc;
    HIPCHK(xf.out(out, dc, bytes));
  }
  return xf.end(async);
}
int mpcekf_lin_fields(mpcekf_ctx *X, const int32_t *slots, int32_t nslots, const double *set, double *out) {
  return lin_fields_impl(X, slots, nslots, set, out, false);
}
int mpcekf_lin_fields_async(mpcekf_ctx *X, const int32_t *slots, int32_t nslots, const double *set, double *out) {
  return lin_fields_impl(X, slots, nslots, set, out, true);
}

int mpcekf_mpc_step(mpcekf_ctx *X, const double *lin, const double *soc_k1, double *uk, int32_t *nexec) {
  return mpcekf_mpc_step_ex(X, lin, soc_k1, uk, nexec, nullptr, nullptr, nullptr, nullptr);
}
int mpcekf_mpc_step_async(mpcekf_ctx *X, const double *lin, const double *soc_k1, double *uk, int32_t *nexec) {
  return mpcekf_mpc_step_ex_async(X, lin, soc_k1, uk, nexec, nullptr, nullptr, nullptr, nullptr);
}

static int mpc_step_ex_impl(mpcekf_ctx *X, const double *lin, const double *soc_k1, double *uk, int32_t *nexec,
                       double *J_unc, double *J_fin, double *norm_du, int32_t *nviol, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!uk) return fail(MPCEKF_E_ARG, "mpc_step: null argument");
  if (!lin && !X->stage_lin) return fail(MPCEKF_E_STATE, "mpc_step: NULL lin but no mpcekf_linearize record");
  if (!soc_k1 && !X->stage_zk) return fail(MPCEKF_E_STATE, "mpc_step: NULL soc_k1 but no mpcekf_ekf_step zk");
  size_t n = (size_t)X->n;
  if ((rc = X->tmp((n * MPCEKF_LIN_SIZE + 5 * n) * 8 + 2 * n * 4 + 4096))) return rc;
  Slab sl{(char *)X->d_tmp};
  double *dl = sl.take<double>(n * MPCEKF_LIN_SIZE), *ds = sl.take<double>(n), *du = sl.take<double>(n);
  double *dju = sl.take<double>(n), *djf = sl.take<double>(n), *dnd = sl.take<double>(n);
  int *dn = sl.take<int>(n), *dv = sl.take<int>(n);
  Xfer xf{X};
  if ((rc = xf.reserve({n * MPCEKF_LIN_SIZE * 8, n * 8, n * 8, n * 8, n * 8, n * 8, n * 4, n * 4}))) return rc;
  if (lin) HIPCHK(xf.in(dl, lin, n * MPCEKF_LIN_SIZE * 8));
  else dl = X->d_slin;  // the device-resident record of the last mpcekf_linearize
  if (soc_k1) HIPCHK(xf.in(ds, soc_k1, n * 8));
  else if ((rc = lerr(launch_cols(X->d_szk, X->n, X->nz + 2, X->d_zslot, 1, ds, false, X->stream), "cols")))
    return rc;  // runMPC.m:99 mpcData.SOCk_1 = zk(end), from the last mpcekf_ekf_step's device zk
  KIO io{};
  io.mode = MODE_MPC;
  io.lin_in = dl;
  io.soc_k1_in = ds;
  io.uk_out = du;
  io.nexec = dn;
  // iterMPC.m:89-95's cost log (mpcData.cost) of this call
  io.junc_out = J_unc ? dju : nullptr;
  io.jfin_out = J_fin ? djf : nullptr;
  io.normdu_out = norm_du ? dnd : nullptr;
  io.nviol_out = nviol ? dv : nullptr;
  if (X->wide) {
    if ((rc = lerr(launch_mpc_wide(X->k, X->s, io, X->w, X->stream), "mpc_wide"))) return rc;
    if ((rc = lerr(launch_hild_wide(X->k, X->s, io, X->w, X->stream), "hild_wide"))) return rc;
  } else {
    if ((rc = lerr(launch_cell(X->r, X->k, X->s, io, X->stream), "cell"))) return rc;
    if ((rc = lerr(launch_hild(X->k, X->s, io, X->stream), "hild"))) return rc;
  }
  HIPCHK(xf.out(uk, du, n * 8));
  if (nexec) HIPCHK(xf.out(nexec, dn, n * 4));
  if (J_unc) HIPCHK(xf.out(J_unc, dju, n * 8));
  if (J_fin) HIPCHK(xf.out(J_fin, djf, n * 8));
  if (norm_du) HIPCHK(xf.out(norm_du, dnd, n * 8));
  if (nviol) HIPCHK(xf.out(nviol, dv, n * 4));
  return xf.end(async);
}
int mpcekf_mpc_step_ex(mpcekf_ctx *X, const double *lin, const double *soc_k1, double *uk, int32_t *nexec,
                       double *J_unc, double *J_fin, double *norm_du, int32_t *nviol) {
  return mpc_step_ex_impl(X, lin, soc_k1, uk, nexec, J_unc, J_fin, norm_du, nviol, false);
}
int mpcekf_mpc_step_ex_async(mpcekf_ctx *X, const double *lin, const double *soc_k1, double *uk, int32_t *nexec,
                       double *J_unc, double *J_fin, double *norm_du, int32_t *nviol) {
  return mpc_step_ex_impl(X, lin, soc_k1, uk, nexec, J_unc, J_fin, norm_du, nviol, true);
}

static int mpc_diag_impl(mpcekf_ctx *X, const double *lin, const double *uk_1, double *poles, double *sv, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!lin && !X->stage_lin) return fail(MPCEKF_E_STATE, "mpc_diag: NULL lin but no mpcekf_linearize record");
  if (!poles && !sv) return MPCEKF_OK;
  size_t n = (size_t)X->n;
  if ((rc = X->tmp((n * MPCEKF_LIN_SIZE + n + n * 3 * NA) * 8 + 2048))) return rc;
  Slab sl{(char *)X->d_tmp};
  double *dl = sl.take<double>(n * MPCEKF_LIN_SIZE), *du = sl.take<double>(n), *dp = sl.take<double>(n * 2 * NA),
         *ds = sl.take<double>(n * NA);
  Xfer xf{X};
  if ((rc = xf.reserve({n * MPCEKF_LIN_SIZE * 8, n * 8, n * 2 * NA * 8, n * NA * 8})))
    return rc;
  if (lin) HIPCHK(xf.in(dl, lin, n * MPCEKF_LIN_SIZE * 8));
  else dl = X->d_slin;
  if (uk_1) HIPCHK(xf.in(du, uk_1, n * 8));
  else HIPCHK(hipMemcpyAsync(du, X->s.uk_1, n * 8, hipMemcpyDeviceToDevice, X->stream));
  rc = X->wide ? launch_cl_diag_wide(X->k, X->n, dl, du, poles ? dp : nullptr, sv ? ds : nullptr, X->stream)
               : launch_cl_diag(X->k, X->n, dl, du, poles ? dp : nullptr, sv ? ds : nullptr, X->stream);
  if ((rc = lerr(rc, "cl_diag"))) return rc;
  if (poles) HIPCHK(xf.out(poles, dp, n * 2 * NA * 8));
  if (sv) HIPCHK(xf.out(sv, ds, n * NA * 8));
  return xf.end(async);
}
int mpcekf_mpc_diag(mpcekf_ctx *X, const double *lin, const double *uk_1, double *poles, double *sv) {
  return mpc_diag_impl(X, lin, uk_1, poles, sv, false);
}
int mpcekf_mpc_diag_async(mpcekf_ctx *X, const double *lin, const double *uk_1, double *poles, double *sv) {
  return mpc_diag_impl(X, lin, uk_1, poles, sv, true);
}

// ---- context-free kernels ----------------------------------------------------
}  // extern "C"
namespace {
struct DevScope {
  hipStream_t st = nullptr;
  char *buf = nullptr;
  ~DevScope() {
    if (st) (void)hipStreamSynchronize(st);
    if (buf) (void)hipFree(buf);
    if (st) (void)hipStreamDestroy(st);
  }
};
}  // namespace
extern "C" {

int mpcekf_predmat(int device, int64_t n, int32_t Np, int32_t Nc, const double *a, const double *C, const double *D,
                   double *Phi, double *G) {
  if (n < 0 || (n && (!a || !C || !D || !Phi || !G))) return fail(MPCEKF_E_ARG, "predmat: bad argument");
  const bool wide = wide_supported(Np, Nc);
  if (!(Np == 5 && Nc == 2) && !wide) return fail(MPCEKF_E_UNSUPPORTED, "predmat: built for Np/Nc = 5/2 and 20/10");
  if (n == 0) return MPCEKF_OK;
  HIPCHK(hipSetDevice(device));
  DevScope d;
  HIPCHK(hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking));
  size_t b_in = (size_t)n * 13 * 8, b_out = (size_t)n * (Np * 7 + Np * Nc) * 8;
  HIPCHK(hipMalloc((void **)&d.buf, b_in + b_out + 1024));
  double *da = (double *)d.buf, *dC = da + n * 6, *dD = dC + n * 6, *dP = dD + n, *dG = dP + n * Np * 7;
  HIPCHK(hipMemcpyAsync(da, a, n * 6 * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dC, C, n * 6 * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dD, D, n * 8, hipMemcpyHostToDevice, d.st));
  int rc = lerr(wide ? launch_predmat_wide(n, Np, Nc, da, dC, dD, dP, dG, d.st)
                     : launch_predmat(n, Np, Nc, da, dC, dD, dP, dG, d.st), "predmat");
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(Phi, dP, n * Np * 7 * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipMemcpyAsync(G, dG, n * Np * Nc * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipStreamSynchronize(d.st));
  return MPCEKF_OK;
}

int mpcekf_constraints(int device, const mpcekf_config *cfg, double Q, int64_t n, const double *lin,
                       const double *uk_1, const double *soc_k1, double *M, double *gamma) {
  if (!cfg || n < 0 || (n && (!lin || !uk_1 || !soc_k1 || !M || !gamma)))
    return fail(MPCEKF_E_ARG, "constraints: bad argument");
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n == 0) return MPCEKF_OK;
  KCfg k{};
  fill_kcfg(cfg, Q, k);
  HIPCHK(hipSetDevice(device));
  DevScope d;
  HIPCHK(hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking));
  const int ncon = ncon_of(cfg->Np, cfg->Nc), Nc = cfg->Nc;
  HIPCHK(hipMalloc((void **)&d.buf, (size_t)n * (MPCEKF_LIN_SIZE + 2 + ncon * Nc + ncon) * 8 + 1024));
  double *dl = (double *)d.buf, *du = dl + n * MPCEKF_LIN_SIZE, *ds = du + n, *dM = ds + n, *dg = dM + n * ncon * Nc;
  HIPCHK(hipMemcpyAsync(dl, lin, n * MPCEKF_LIN_SIZE * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(du, uk_1, n * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(ds, soc_k1, n * 8, hipMemcpyHostToDevice, d.st));
  if ((rc = lerr(wide_supported(cfg->Np, Nc) ? launch_constraints_wide(k, cfg->Np, Nc, n, dl, du, ds, dM, dg, d.st)
                                               : launch_constraints(k, n, dl, du, ds, dM, dg, d.st),
                 "constraints")))
    return rc;
  HIPCHK(hipMemcpyAsync(M, dM, n * ncon * Nc * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipMemcpyAsync(gamma, dg, n * ncon * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipStreamSynchronize(d.st));
  return MPCEKF_OK;
}

int mpcekf_hildreth(int device, int64_t n, int32_t Nc, int32_t ncon, const double *E, const double *F,
                    const double *M, const double *gamma, double *lambda, int32_t max_iter, double tol, double *DU,
                    int32_t *nexec) {
  if (n < 0 || (n && (!E || !F || !M || !gamma || !lambda || !DU || !nexec)))
    return fail(MPCEKF_E_ARG, "hildreth: bad argument");
  if (Nc < 1 || Nc > 10 || ncon < 1 || ncon > 100)
    return fail(MPCEKF_E_UNSUPPORTED, "hildreth: Nc must be 1..10 and the constraint count 1..100");
  if (max_iter < 1) return fail(MPCEKF_E_ARG, "hildreth: max_iter < 1");
  if (n == 0) return MPCEKF_OK;
  HIPCHK(hipSetDevice(device));
  DevScope d;
  HIPCHK(hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking));
  size_t per = (size_t)(Nc * Nc + Nc + ncon * Nc + ncon + ncon + Nc);
  const bool any = Nc != 2 || ncon != NCON_BUILT;
  const size_t scr = any ? hildreth_any_scratch(n, Nc, ncon) : 0;
  HIPCHK(hipMalloc((void **)&d.buf, (size_t)n * per * 8 + (size_t)n * 4 + scr * 8 + 1024));
  double *dE = (double *)d.buf, *dF = dE + n * Nc * Nc, *dM = dF + n * Nc, *dg = dM + n * ncon * Nc,
         *dl = dg + n * ncon, *dD = dl + n * ncon;
  int *dn = (int *)(dD + n * Nc);
  HIPCHK(hipMemcpyAsync(dE, E, n * Nc * Nc * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dF, F, n * Nc * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dM, M, n * ncon * Nc * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dg, gamma, n * ncon * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dl, lambda, n * ncon * 8, hipMemcpyHostToDevice, d.st));
  double *dscr = any ? (double *)(((uintptr_t)(dn + n) + 255) & ~(uintptr_t)255) : nullptr;
  int rc = lerr(launch_hildreth(n, Nc, ncon, dE, dF, dM, dg, dl, max_iter, tol, dD, dn, d.st, dscr), "hildreth");
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(lambda, dl, n * ncon * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipMemcpyAsync(DU, dD, n * Nc * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipMemcpyAsync(nexec, dn, n * 4, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipStreamSynchronize(d.st));
  return MPCEKF_OK;
}

int mpcekf_hildreth_structured(int device, int64_t n, const double *E, const double *F, const double *Hv,
                               const double *He, const double *Hs, const double *gamma, double *lambda,
                               int32_t max_iter, double tol, double *DU, int32_t *nexec) {
  if (n < 0 || (n && (!E || !F || !Hv || !He || !Hs || !gamma || !lambda || !DU || !nexec)))
    return fail(MPCEKF_E_ARG, "hildreth_structured: bad argument");
  if (max_iter < 1) return fail(MPCEKF_E_ARG, "hildreth_structured: max_iter < 1");
  if (n == 0) return MPCEKF_OK;
  HIPCHK(hipSetDevice(device));
  DevScope d;
  HIPCHK(hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking));
  const size_t NCn = 2, NPn = 5, NCONn = NCON_BUILT;
  const size_t per = NCn * NCn + NCn + 3 * NPn + NCONn + NCONn + NCn;
  HIPCHK(hipMalloc((void **)&d.buf, (size_t)n * per * 8 + (size_t)n * 4 + 1024));
  double *dE = (double *)d.buf, *dF = dE + n * NCn * NCn, *dHv = dF + n * NCn, *dHe = dHv + n * NPn,
         *dHs = dHe + n * NPn, *dg = dHs + n * NPn, *dl = dg + n * NCONn, *dD = dl + n * NCONn;
  int *dn = (int *)(dD + n * NCn);
  HIPCHK(hipMemcpyAsync(dE, E, n * NCn * NCn * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dF, F, n * NCn * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dHv, Hv, n * NPn * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dHe, He, n * NPn * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dHs, Hs, n * NPn * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dg, gamma, n * NCONn * 8, hipMemcpyHostToDevice, d.st));
  HIPCHK(hipMemcpyAsync(dl, lambda, n * NCONn * 8, hipMemcpyHostToDevice, d.st));
  int rc = lerr(launch_hildreth_structured(n, dE, dF, dHv, dHe, dHs, dg, dl, max_iter, tol, dD, dn, d.st),
                "hildreth_structured");
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(lambda, dl, n * NCONn * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipMemcpyAsync(DU, dD, n * NCn * 8, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipMemcpyAsync(nexec, dn, n * 4, hipMemcpyDeviceToHost, d.st));
  HIPCHK(hipStreamSynchronize(d.st));
  return MPCEKF_OK;
}

int mpcekf_get_hild_problems(mpcekf_ctx *X, double *prob, int32_t *hflag) {
  int rc = need_init(X);
  if (rc) return rc;
  static_assert(MPCEKF_PROB_DOUBLES == PROB_DOUBLES, "problem record size");
  if (X->wide) return fail(MPCEKF_E_UNSUPPORTED, "get_hild_problems: Np = 5 / Nc = 2 records only");
  const size_t n = (size_t)X->n;
  if (prob) HIPCHK(hipMemcpyAsync(prob, X->s.prob, n * PROB_DOUBLES * 8, hipMemcpyDeviceToHost, X->stream));
  if (hflag) HIPCHK(hipMemcpyAsync(hflag, X->s.hflag, n * 4, hipMemcpyDeviceToHost, X->stream));
  HIPCHK(hipStreamSynchronize(X->stream));
  return MPCEKF_OK;
}

int mpcekf_get_stamps(mpcekf_ctx *X, int64_t *stamps, int32_t *nstamps) {
  int rc = need_init(X);
  if (rc) return rc;
  static_assert(MPCEKF_NSTAMPS == NSTAMPS, "stamp count");
  if (nstamps) *nstamps = X->d_stamps ? NSTAMPS : 0;
  if (X->d_stamps && stamps) {
    HIPCHK(hipMemcpyAsync(stamps, X->d_stamps, (size_t)X->n * NSTAMPS * 8, hipMemcpyDeviceToHost, X->stream));
    HIPCHK(hipStreamSynchronize(X->stream));
  }
  return MPCEKF_OK;
}

// ---- state access ------------------------------------------------------------
static const int kScalMap[MPCEKF_NSCAL] = {0, 1, 2, 3, 4, 5, 6, 7};  // MPCEKF_S_* -> d_scal slot

int mpcekf_get_state(mpcekf_ctx *X, mpcekf_state *st) {
  int rc = need_init(X);
  if (rc) return rc;
  if (!st) return fail(MPCEKF_E_ARG, "get_state: null");
  const size_t n = (size_t)X->n, NM = (size_t)X->NM, nc = (size_t)X->ncon;
  if (st->bigX) HIPCHK(hipMemcpyAsync(st->bigX, X->s.bigx, n * NM * 6 * 8, hipMemcpyDeviceToHost, X->stream));
  if (st->ekf) HIPCHK(hipMemcpyAsync(st->ekf, X->s.ekf, n * NM * REC * 8, hipMemcpyDeviceToHost, X->stream));
  if (st->mb && X->mb) HIPCHK(hipMemcpyAsync(st->mb, X->d_mb, n * MBREC * 8, hipMemcpyDeviceToHost, X->stream));
  // only the requested fields cross PCIe (a MEX drop-in reading SOCnAvg/SOCpAvg each
  // step moves the 64-B scalar block per cell, not the NM-model records)
  std::vector<double> sc(st->scal ? n * 8 : 0), lam(st->lambda ? n * nc : 0);
  std::vector<int> iv(st->warn || st->status ? n * 2 : 0);
  if (st->scal) HIPCHK(hipMemcpyAsync(sc.data(), X->d_scal, n * 8 * 8, hipMemcpyDeviceToHost, X->stream));
  if (st->lambda) HIPCHK(hipMemcpyAsync(lam.data(), X->s.lam, n * nc * 8, hipMemcpyDeviceToHost, X->stream));
  if (!iv.empty()) HIPCHK(hipMemcpyAsync(iv.data(), X->d_int, n * 2 * 4, hipMemcpyDeviceToHost, X->stream));
  HIPCHK(hipStreamSynchronize(X->stream));
  for (size_t c = 0; c < n; ++c) {
    if (st->scal)
      for (int k = 0; k < MPCEKF_NSCAL; ++k) st->scal[c * MPCEKF_NSCAL + k] = sc[kScalMap[k] * n + c];
    if (st->lambda)
      for (size_t i = 0; i < nc; ++i) st->lambda[c * nc + i] = lam[i * n + c];
    if (st->warn) st->warn[c] = iv[c];
    if (st->status) st->status[c] = iv[n + c];
  }
  return MPCEKF_OK;
}

static int get_scalars_impl(mpcekf_ctx *X, const int32_t *slots, int32_t nslots, double *scal, int32_t *warn,
                            int32_t *status, bool async) {
  int rc = need_init(X);
  if (rc) return rc;
  if (nslots < 0 || nslots > MPCEKF_NSCAL || (nslots && (!slots || !scal)))
    return fail(MPCEKF_E_ARG, "get_scalars: bad slot list");
  for (int j = 0; j < nslots; ++j)
    if (slots[j] < 0 || slots[j] >= MPCEKF_NSCAL) return fail(MPCEKF_E_ARG, "get_scalars: slot %d", slots[j]);
  const size_t n = (size_t)X->n;
  // the SoA scalar block holds each slot as one contiguous [ncells] vector; a gather kernel
  // (k_rows) lays the requested ones out cell-major, so exactly those bytes cross PCIe in one
  // copy and the host does no transposition (nor the _async form at its synchronisation)
  int rows[MPCEKF_NSCAL];
  for (int j = 0; j < nslots; ++j) rows[j] = kScalMap[slots[j]];
  if ((rc = X->tmp(n * (size_t)nslots * 8 + 1024))) return rc;
  Slab sl{(char *)X->d_tmp};
  double *dc = sl.take<double>(n * (size_t)nslots);
  int *dr = sl.take<int>(MPCEKF_NSCAL);
  Xfer xf{X};
  if ((rc = xf.reserve({sizeof rows, n * (size_t)nslots * 8, n * 4, n * 4}))) return rc;
  if (nslots) {
    HIPCHK(xf.in(dr, rows, (size_t)nslots * sizeof(int)));
    if ((rc = lerr(launch_rows(X->d_scal, X->n, dr, nslots, dc, X->stream), "rows"))) return rc;
    HIPCHK(xf.out(scal, dc, n * (size_t)nslots * 8));
  }
  if (warn) HIPCHK(xf.out(warn, X->s.warn, n * 4));
  if (status) HIPCHK(xf.out(status, X->s.status, n * 4));
  return xf.end(async);
}
int mpcekf_get_scalars(mpcekf_ctx *X, const int32_t *slots, int32_t nslots, double *scal, int32_t *warn,
                       int32_t *status) {
  return get_scalars_impl(X, slots, nslots, scal, warn, status, false);
}
int mpcekf_get_scalars_async(mpcekf_ctx *X, const int32_t *slots, int32_t nslots, double *scal, int32_t *warn,
                             int32_t *status) {
  return get_scalars_impl(X, slots, nslots, scal, warn, status, true);
}

int mpcekf_set_state(mpcekf_ctx *X, const mpcekf_state *st) {
  if (X) X->stage_zk = X->stage_lin = X->stage_v = false;  // the stage route's device hand-offs are stale
  int rc = need_init(X);
  if (rc) return rc;
  if (!st) return fail(MPCEKF_E_ARG, "set_state: null");
  const size_t n = (size_t)X->n, NM = (size_t)X->NM, nc = (size_t)X->ncon;
  if (st->bigX) HIPCHK(hipMemcpyAsync(X->s.bigx, st->bigX, n * NM * 6 * 8, hipMemcpyHostToDevice, X->stream));
  if (st->ekf) HIPCHK(hipMemcpyAsync(X->s.ekf, st->ekf, n * NM * REC * 8, hipMemcpyHostToDevice, X->stream));
  if (st->mb && X->mb) HIPCHK(hipMemcpyAsync(X->d_mb, st->mb, n * MBREC * 8, hipMemcpyHostToDevice, X->stream));
  // scal and lambda are whole blocks (every slot given); warn and status share one block,
  // read back first when only one of them is given
  std::vector<double> sc(st->scal ? n * 8 : 0), lam(st->lambda ? n * nc : 0);
  std::vector<int> iv(st->warn || st->status ? n * 2 : 0);
  if (!iv.empty() && !(st->warn && st->status)) {
    HIPCHK(hipMemcpyAsync(iv.data(), X->d_int, n * 2 * 4, hipMemcpyDeviceToHost, X->stream));
    HIPCHK(hipStreamSynchronize(X->stream));
  }
  for (size_t c = 0; c < n; ++c) {
    if (st->scal)
      for (int k = 0; k < MPCEKF_NSCAL; ++k) sc[kScalMap[k] * n + c] = st->scal[c * MPCEKF_NSCAL + k];
    if (st->lambda)
      for (size_t i = 0; i < nc; ++i) lam[i * n + c] = st->lambda[c * nc + i];
    if (st->warn) iv[c] = st->warn[c];
    if (st->status) iv[n + c] = st->status[c];
  }
  if (st->scal) HIPCHK(hipMemcpyAsync(X->d_scal, sc.data(), n * 8 * 8, hipMemcpyHostToDevice, X->stream));
  if (st->lambda) HIPCHK(hipMemcpyAsync(X->s.lam, lam.data(), n * nc * 8, hipMemcpyHostToDevice, X->stream));
  if (!iv.empty()) HIPCHK(hipMemcpyAsync(X->d_int, iv.data(), n * 2 * 4, hipMemcpyHostToDevice, X->stream));
  HIPCHK(hipStreamSynchronize(X->stream));
  return MPCEKF_OK;
}

}  // extern "C"
