/* The drop-ins' stage sequence (the matlab/dropin wrappers on the device route: OB_step -> iterEKF ->
 * EKFmatsHandler (records kept on the device) -> lin_fields -> mpc_diag -> iterMPC, with the
 * per-step scalars the wrappers read) driven from C through the C-ABI, as a MEX host would
 * drive it: every output array is freshly malloc'ed for its call and freed after the step,
 * like MATLAB's mxArrays.  tools/dropin_bench.py --route c / c-async calls dropin_loop through
 * ctypes on a context it created, so this times the library route without the Python
 * binding's per-call work.  Host code only; built by tools/dropin_bench.py with gcc.
 *
 * mode bit 0 (async): every stage but iterMPC through its _async twin (Vcell and zk(end) handed
 * over on the device: vk = NULL, soc_k1 = NULL), iterMPC synchronous -- one synchronisation per
 * step.  Bit 1 (reuse): the output arrays are allocated once and reused by every step, as a host
 * that keeps its buffers (or an allocator that hands the same pages back) would; without it each
 * step pays the caller's allocator: fresh pages faulted in by the copies, unmapped at free. */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpcekf.h"

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

enum { ST_SCAL, ST_PLANT, ST_EKF, ST_LIN, ST_FIELDS, ST_DIAG, ST_MPC, NST };

/* scal_a / scal_b: the scalar slots read before the plant and after iterEKF (OB_step.m:226-228,
 * the ekfData fields); fields: the lin_fields slots (runMPC.m:95-96).  uk [n] in: the first
 * command; out: the last.  ms [NST]: per-stage milliseconds summed over the timed steps;
 * bytes: host bytes moved per cell-step.  Returns 0 or the first failing call's code. */
int dropin_loop(mpcekf_ctx *ctx, int64_t n, int32_t nz, int32_t steps, int32_t warmup, int32_t mode,
                const double *tc, const int32_t *scal_a, int32_t nscal_a, const int32_t *scal_b, int32_t nscal_b,
                const int32_t *fields, int32_t nfields, double *uk, double *ms, double *ms_total, double *bytes) {
  const size_t N = (size_t)n, NZ2 = (size_t)nz + 2;
  const int async = mode & 1, reuse = (mode >> 1) & 1;
  double *u = malloc(N * 8);
  if (!u) return -1;
  memcpy(u, uk, N * 8);
  for (int k = 0; k < NST; ++k) ms[k] = 0.0;
  double t_start = 0.0, b = 0.0;
  int rc = 0;
  double *sa = NULL, *v = NULL, *zk = NULL, *zb = NULL, *xg = NULL, *sb = NULL, *f = NULL, *poles = NULL, *sv = NULL;
  double *un = NULL, *ju = NULL, *jf = NULL, *nd = NULL, *socm = NULL;
  int32_t *xm = NULL, *warn = NULL, *status = NULL, *ne = NULL, *nv = NULL;
  for (int s = 0; s < warmup + steps && !rc; ++s) {
    const int timed = s >= warmup;
    if (s == warmup) t_start = now_ms();
    double t0, t1;
#define STAGE(id, call)              \
  do {                               \
    t0 = now_ms();                   \
    rc = (call);                     \
    t1 = now_ms();                   \
    if (timed) ms[id] += t1 - t0;    \
    if (rc) goto step_end;           \
  } while (0)
    if (!reuse || !sa) {
      sa = malloc(N * nscal_a * 8); v = malloc(N * 8); zk = malloc(N * NZ2 * 8); zb = malloc(N * NZ2 * 8);
      xm = malloc(N * 4 * 4); xg = malloc(N * 4 * 8); sb = malloc(N * nscal_b * 8);
      warn = malloc(N * 4); status = malloc(N * 4);
      f = malloc(N * nfields * 8); poles = malloc(N * 14 * 8); sv = malloc(N * 7 * 8);
      un = malloc(N * 8); ju = malloc(N * 8); jf = malloc(N * 8); nd = malloc(N * 8); socm = malloc(N * 8);
      ne = malloc(N * 4); nv = malloc(N * 4);
    }
    if (!sa || !v || !zk || !zb || !xm || !xg || !sb || !warn || !status || !f || !poles || !sv || !un || !ju || !jf ||
        !nd || !socm || !ne || !nv) {
      rc = -1;
      goto step_end;
    }
    if (async) {
      STAGE(ST_SCAL, mpcekf_get_scalars_async(ctx, scal_a, nscal_a, sa, NULL, NULL));
      STAGE(ST_PLANT, mpcekf_plant_step_async(ctx, u, tc, v));
      STAGE(ST_EKF, mpcekf_ekf_step_async(ctx, NULL, u, tc, zk, zb, xm, xg));
      STAGE(ST_SCAL, mpcekf_get_scalars_async(ctx, scal_b, nscal_b, sb, warn, status));
      STAGE(ST_LIN, mpcekf_linearize_async(ctx, NULL, NULL, NULL, tc, NULL));
      STAGE(ST_FIELDS, mpcekf_lin_fields_async(ctx, fields, nfields, NULL, f));
      STAGE(ST_DIAG, mpcekf_mpc_diag_async(ctx, NULL, NULL, poles, sv));
      STAGE(ST_MPC, mpcekf_mpc_step_ex(ctx, NULL, NULL, un, ne, ju, jf, nd, nv));
    } else {
      STAGE(ST_SCAL, mpcekf_get_scalars(ctx, scal_a, nscal_a, sa, NULL, NULL));
      STAGE(ST_PLANT, mpcekf_plant_step(ctx, u, tc, v));
      STAGE(ST_EKF, mpcekf_ekf_step(ctx, v, u, tc, zk, zb, xm, xg));
      STAGE(ST_SCAL, mpcekf_get_scalars(ctx, scal_b, nscal_b, sb, warn, status));
      STAGE(ST_LIN, mpcekf_linearize(ctx, NULL, NULL, NULL, tc, NULL));
      STAGE(ST_FIELDS, mpcekf_lin_fields(ctx, fields, nfields, NULL, f));
      STAGE(ST_DIAG, mpcekf_mpc_diag(ctx, NULL, NULL, poles, sv));
      for (size_t c = 0; c < N; ++c) socm[c] = zk[c * NZ2 + NZ2 - 1];  /* zk(end,:) */
      STAGE(ST_MPC, mpcekf_mpc_step_ex(ctx, NULL, socm, un, ne, ju, jf, nd, nv));
    }
#undef STAGE
    memcpy(u, un, N * 8);
    if (timed) /* per cell: scalars; plant iapp, tc in, V out; ekf (vk,) ik, tk in, zk, boundzk, Xind out;
                  scalars + warn / status; linearize tk; lin_fields; poles / sv; iterMPC (soc_k1,) out */
      b += (double)(nscal_a * 8 + 24 + (async ? 16 : 24) + (16 * NZ2 + 48) + (nscal_b * 8 + 8) + 8 + nfields * 8 +
                    168 + (async ? 0 : 8) + 40);
  step_end:
    if (!reuse || rc || s + 1 == warmup + steps) {
      free(sa); free(v); free(zk); free(zb); free(xm); free(xg); free(sb); free(warn); free(status); free(f);
      free(poles); free(sv); free(un); free(ju); free(jf); free(nd); free(socm); free(ne); free(nv);
      sa = NULL;
    }
  }
  *ms_total = now_ms() - t_start;
  *bytes = steps ? b / steps : 0.0;
  memcpy(uk, u, N * 8);
  free(u);
  return rc;
}
