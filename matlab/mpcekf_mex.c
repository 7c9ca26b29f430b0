/*
 * mpcekf_mex.c -- MEX gateway from MATLAB to the MI355X library (include/mpcekf.h).
 *
 * Build (on a machine with MATLAB and the built library; not buildable in this
 * repository's container, which has no MATLAB):
 *   mex -R2018a -I../include mpcekf_mex.c -L../mpc-ekf4fastcharge_amd/_build -lmpcekf
 *
 * One command string per C-ABI entry point, the context kept as a uint64 handle:
 *   h                 = mpcekf_mex('create', R, cfg, device, ncells)   mpcekf_ctx_create
 *                       R: struct from mpcekf_rom_struct(ROM); cfg: struct of mpcekf_config
 *                       fields (missing fields keep the runMPC.m defaults)
 *                       mpcekf_mex('destroy', h)                       mpcekf_ctx_destroy
 *                       mpcekf_mex('init', h, soc0_pct, tc_degC)       mpcekf_init_cells
 *   [u,v,soc,phise,nexec] = mpcekf_mex('step', h, nsteps, tc)          mpcekf_step
 *                       tc: [] or ncells x nsteps (degC); outputs ncells x nsteps
 *   v                 = mpcekf_mex('plant', h, iapp, tc)               mpcekf_plant_step   (OB_step.m:1)
 *   [zk,zbk,xm,xg]    = mpcekf_mex('ekf', h, vk, ik, tk)               mpcekf_ekf_step     (iterEKF.m:30)
 *   lin               = mpcekf_mex('linearize', h, zk, xm, xg, tk)     mpcekf_linearize    (EKFmatsHandler.m:1)
 *   [uk,nexec,J_uncon,J_final,norm_DU,viol] = mpcekf_mex('mpc', h, lin, soc_k1)
 *                                                                      mpcekf_mpc_step_ex  (iterMPC.m:1,89-95)
 *   [poles,sv]        = mpcekf_mex('mpcdiag', h, lin, uk_1)            mpcekf_mpc_diag     (iterMPC.m:53-60)
 *                       uk_1: [] for the context's; poles complex 7 x ncells, sv 7 x ncells
 *   [DU,lambda,nexec] = mpcekf_mex('hildreth', E, F, M, gamma, lambda0, maxIter)   (hildreth.m:1)
 *   [Phi,G]           = mpcekf_mex('predmat', a, C, D, Np, Nc)         (predMat.m:1, A = diag(a), B = 1)
 *   st                = mpcekf_mex('get_state', h)    /  mpcekf_mex('set_state', h, st)
 *                       st.bigX, ekf, scal, lambda (double), warn, status (int32 1 x ncells),
 *                       and st.mb (42 x ncells) on a model-blend ('MB') context (optional
 *                       in set_state: a checkpoint without it keeps the blend state)
 *   [s,warn,status]   = mpcekf_mex('scalars', h, idx)                 mpcekf_get_scalars
 *                       s: numel(idx) x ncells of the 1-based MPCEKF_S_* slots idx (1-2
 *                       SOCnAvg/SOCpAvg, 3 x0, 4 SigmaX0, 5 priorI, 6 uk_1, 7 uk, 8 vk):
 *                       what the drop-ins read every step, 8 B per slot and cell
 *                       mpcekf_mex('graph', h, enable)                 mpcekf_set_graph (replay repeated step calls)
 * Per-cell vectors are 1 x ncells or ncells x 1; zk / zbk are (nz+2) x ncells, xm / xg
 * 4 x ncells (xm: 0-based model index t*nZ+z), lin 35 x ncells -- MATLAB's column-major
 * k x ncells is the library's cell-major [ncells][k], so no copy is made for them.
 * Arrays the library reads row-major (the ROM's A/C/D, the electrode tables, hildreth's
 * E and M) are transposed here from MATLAB's column-major order.
 * Scalars (device, ncells, nsteps, cfg fields ...) may be of any real numeric class.
 * Only the first max(nargout, 1) outputs are returned.
 * Library failures raise a MATLAB error with mpcekf_last_error(); per-cell soft
 * failures stay in the status word (get_state), as in the C-ABI.
 * `clear mex` / MATLAB exit destroys every context still live (mexAtExit), freeing its
 * device memory; handles saved across a clear are then rejected as not live.
 */
#include <stdint.h>
#include <string.h>

#include "matrix.h"
#include "mex.h"
#include "mpcekf.h"

static void chk(int rc) {
  if (rc != MPCEKF_OK) mexErrMsgIdAndTxt("mpcekf:lib", "mpcekf error %d: %s", rc, mpcekf_last_error());
}

/* Live contexts of this MEX session: a handle is checked against them before use, so a
 * stale or made-up uint64 raises a MATLAB error instead of crashing MATLAB. */
#define MAXCTX 64
static mpcekf_ctx *g_live[MAXCTX];

static void track(mpcekf_ctx *h, int add) {
  for (int i = 0; i < MAXCTX; ++i)
    if (add ? g_live[i] == NULL : g_live[i] == h) {
      g_live[i] = add ? h : NULL;
      return;
    }
}

/* mexAtExit: `clear mex` or MATLAB exit releases every live context's device memory */
static void destroy_all(void) {
  for (int i = 0; i < MAXCTX; ++i)
    if (g_live[i]) {
      (void)mpcekf_ctx_destroy(g_live[i]);
      g_live[i] = NULL;
    }
}

static mpcekf_ctx *handle(const mxArray *a) {
  if (!mxIsUint64(a) || mxGetNumberOfElements(a) != 1) mexErrMsgIdAndTxt("mpcekf:arg", "expected a uint64 handle");
  mpcekf_ctx *h = (mpcekf_ctx *)(uintptr_t)(*(uint64_t *)mxGetData(a));
  for (int i = 0; i < MAXCTX; ++i)
    if (h && g_live[i] == h) return h;
  mexErrMsgIdAndTxt("mpcekf:arg", "not a live mpcekf context handle (destroyed, or not from 'create')");
  return NULL;
}

/* a real scalar of any numeric class (double, int32, ...), as MATLAB code passes them */
static double scalar(const mxArray *a, const char *what) {
  if (!a || !mxIsNumeric(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != 1)
    mexErrMsgIdAndTxt("mpcekf:arg", "%s: expected a real numeric scalar", what);
  return mxGetScalar(a);
}

/* an int32 array of exactly n elements (warn / status / xm) */
static int32_t *ivec(const mxArray *a, size_t n, const char *what) {
  if (!a || !mxIsInt32(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != n)
    mexErrMsgIdAndTxt("mpcekf:arg", "%s: expected %zu int32 values", what, n);
  return (int32_t *)mxGetData(a);
}

static const double *dvec(const mxArray *a, size_t n, const char *what) {
  if (!a || !mxIsDouble(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != n)
    mexErrMsgIdAndTxt("mpcekf:arg", "%s: expected %zu real doubles", what, n);
  return mxGetDoubles(a);
}

/* MATLAB column-major N-D array -> C row-major copy (same dims) */
static double *rowmajor(const mxArray *a, const char *what) {
  if (!a || !mxIsDouble(a) || mxIsComplex(a)) mexErrMsgIdAndTxt("mpcekf:arg", "%s: expected a real double array", what);
  const mwSize nd = mxGetNumberOfDimensions(a);
  const mwSize *dims = mxGetDimensions(a);
  const size_t n = mxGetNumberOfElements(a);
  const double *src = mxGetDoubles(a);
  double *dst = (double *)mxMalloc(n * sizeof(double) + 8);
  mwSize idx[8] = {0};
  if (nd > 8) mexErrMsgIdAndTxt("mpcekf:arg", "%s: too many dimensions", what);
  for (size_t lin = 0; lin < n; ++lin) { /* lin walks the row-major order; idx its subscripts */
    size_t cm = 0, stride = 1;
    for (mwSize d = 0; d < nd; ++d) {
      cm += idx[d] * stride;
      stride *= dims[d];
    }
    dst[lin] = src[cm];
    for (mwSize d = nd; d-- > 0;) {
      if (++idx[d] < dims[d]) break;
      idx[d] = 0;
    }
  }
  return dst;
}

static const mxArray *field(const mxArray *s, const char *name) {
  const mxArray *f = mxGetField(s, 0, name);
  if (!f) mexErrMsgIdAndTxt("mpcekf:arg", "struct: missing field %s", name);
  return f;
}

/* ABI v3 (optional): e.poly.{Uocp,dUocp,k0,Rf,Cdleff} ntemp x (ntheta-1) x npoly and
 * e.poly.Uocp1 (ntheta-1) x npoly theta polynomials; e.Ea 1 x 5 Arrhenius energies (J/mol)
 * of Uocp, dUocp, k0, Rf, Cdleff.  Returns npoly (0: no polynomials). */
static int electrode_v3(const mxArray *e, mpcekf_electrode *out, int ntemp, int ntheta) {
  const mxArray *ea = mxGetField(e, 0, "Ea");
  if (ea && !mxIsEmpty(ea)) {
    const double *v = dvec(ea, 5, "Ea");
    for (int i = 0; i < 5; ++i) out->Ea[i] = v[i];
  }
  const mxArray *p = mxGetField(e, 0, "poly");
  if (!p || mxIsEmpty(p)) return 0;
  if (!mxIsStruct(p)) mexErrMsgIdAndTxt("mpcekf:arg", "poly: expected a struct");
  const mxArray *u1 = field(p, "Uocp1");
  const int np = (int)mxGetN(u1);
  if ((np != 4 && np != 6) || mxGetM(u1) != (size_t)(ntheta - 1))
    mexErrMsgIdAndTxt("mpcekf:arg", "poly.Uocp1: expected (ntheta-1) x 4 or x 6");
  out->Uocp1_p = rowmajor(u1, "poly.Uocp1");
  const char *names[5] = {"Uocp", "dUocp", "k0", "Rf", "Cdleff"};
  const double **dst[5] = {&out->Uocp_p, &out->dUocp_p, &out->k0_p, &out->Rf_p, &out->Cdleff_p};
  for (int i = 0; i < 5; ++i) {
    const mxArray *t = field(p, names[i]);
    if (mxGetNumberOfElements(t) != (size_t)ntemp * (ntheta - 1) * np)
      mexErrMsgIdAndTxt("mpcekf:arg", "poly.%s: expected ntemp x (ntheta-1) x %d", names[i], np);
    *dst[i] = rowmajor(t, names[i]);
  }
  return np;
}

/* ABI v4 (optional): e.nodes.{Uocp,dUocp,k0,Rf,Cdleff,Uocp1}, each a struct with x (1 x m
 * ascending theta nodes) and p (ntemp x (m-1) x npoly; Uocp1 (m-1) x npoly) -- a function
 * on its own breakpoints (include/mpcekf.h nnode / node / node_p; mpcekf_build_tables fills
 * them for lookup-table handles).  npoly must be the poly tables' (tab_npoly). */
static void electrode_v4(const mxArray *e, mpcekf_electrode *out, int ntemp, int npoly) {
  const mxArray *nd = mxGetField(e, 0, "nodes");
  if (!nd || mxIsEmpty(nd)) return;
  if (!mxIsStruct(nd)) mexErrMsgIdAndTxt("mpcekf:arg", "nodes: expected a struct");
  if (!npoly) mexErrMsgIdAndTxt("mpcekf:arg", "nodes: needs the poly tables (ABI v3) beside them");
  const char *names[6] = {"Uocp", "dUocp", "k0", "Rf", "Cdleff", "Uocp1"};
  for (int f = 0; f < 6; ++f) {
    const mxArray *t = mxGetField(nd, 0, names[f]);
    if (!t || mxIsEmpty(t)) continue;
    const mxArray *x = field(t, "x"), *p = field(t, "p");
    const size_t m = mxGetNumberOfElements(x);
    const size_t rows = f == 5 ? 1 : (size_t)ntemp;
    if (m < 2 || mxGetNumberOfElements(p) != rows * (m - 1) * (size_t)npoly)
      mexErrMsgIdAndTxt("mpcekf:arg", "nodes.%s: x needs >= 2 nodes and p %s x (m-1) x %d", names[f],
                        f == 5 ? "1" : "ntemp", npoly);
    out->nnode[f] = (int32_t)m;
    out->node[f] = dvec(x, m, names[f]);
    out->node_p[f] = rowmajor(p, names[f]);
  }
}

static void electrode(const mxArray *e, mpcekf_electrode *out, int ntemp, int ntheta) {
  out->theta0 = scalar(field(e, "theta0"), "theta0");
  out->theta100 = scalar(field(e, "theta100"), "theta100");
  out->soc0 = dvec(field(e, "soc0"), (size_t)ntemp, "soc0");
  out->soc100 = dvec(field(e, "soc100"), (size_t)ntemp, "soc100");
  out->Uocp1 = dvec(field(e, "Uocp1"), (size_t)ntheta, "Uocp1");
  const char *names[5] = {"Uocp", "dUocp", "k0", "Rf", "Cdleff"};
  const double **dst[5] = {&out->Uocp, &out->dUocp, &out->k0, &out->Rf, &out->Cdleff};
  for (int i = 0; i < 5; ++i) { /* ntemp x ntheta in MATLAB -> [ntemp][ntheta] */
    const mxArray *t = field(e, names[i]);
    if (mxGetNumberOfElements(t) != (size_t)ntemp * ntheta) mexErrMsgIdAndTxt("mpcekf:arg", "%s: size", names[i]);
    *dst[i] = rowmajor(t, names[i]);
  }
}

static void rom_from_struct(const mxArray *R, mpcekf_rom *r) {
  memset(r, 0, sizeof(*r));
  const mxArray *A = field(R, "A"), *C = field(R, "C");
  const mwSize *da = mxGetDimensions(A), *dc = mxGetDimensions(C);
  if (mxGetNumberOfDimensions(A) != 3 || mxGetNumberOfDimensions(C) != 4)
    mexErrMsgIdAndTxt("mpcekf:arg", "ROM: A must be nT x nZ x (n+1), C nT x nZ x nz x (n+1)");
  r->nT = (int32_t)da[0];
  r->nZ = (int32_t)da[1];
  r->n = (int32_t)da[2] - 1;
  r->nz = (int32_t)dc[2];
  r->T_degC = dvec(field(R, "T_degC"), (size_t)r->nT, "T_degC");
  r->SOC_pct = dvec(field(R, "SOC_pct"), (size_t)r->nZ, "SOC_pct");
  r->Ts = scalar(field(R, "Ts"), "Ts");
  r->A = rowmajor(A, "A");
  r->C = rowmajor(C, "C");
  r->D = rowmajor(field(R, "D"), "D");
  const mxArray *code = field(R, "tf_code");
  if (!mxIsInt32(code) || mxGetNumberOfElements(code) != (size_t)r->nz) mexErrMsgIdAndTxt("mpcekf:arg", "tf_code: int32 x nz");
  r->tf_code = (const int32_t *)mxGetData(code);
  r->tf_xloc = dvec(field(R, "xloc"), (size_t)r->nz, "xloc");
  r->F = scalar(field(R, "F"), "F");
  r->R = scalar(field(R, "R"), "R");
  r->Q = scalar(field(R, "Q"), "Q");
  r->Rc = scalar(field(R, "Rc"), "Rc");
  r->Tref = scalar(field(R, "Tref"), "Tref");
  const mxArray *TK = field(R, "tab_T_K");
  r->tab_ntemp = (int32_t)mxGetNumberOfElements(TK);
  r->tab_T_K = dvec(TK, (size_t)r->tab_ntemp, "tab_T_K");
  r->tab_ntheta = (int32_t)mxGetNumberOfElements(field(field(R, "neg"), "Uocp1"));
  electrode(field(R, "neg"), &r->neg, r->tab_ntemp, r->tab_ntheta);
  electrode(field(R, "pos"), &r->pos, r->tab_ntemp, r->tab_ntheta);
  const int npn = electrode_v3(field(R, "neg"), &r->neg, r->tab_ntemp, r->tab_ntheta);
  const int npp = electrode_v3(field(R, "pos"), &r->pos, r->tab_ntemp, r->tab_ntheta);
  if (npn != npp) mexErrMsgIdAndTxt("mpcekf:arg", "ROM: poly tables for both electrodes or neither, same order");
  r->tab_npoly = npn;
  electrode_v4(field(R, "neg"), &r->neg, r->tab_ntemp, npn);
  electrode_v4(field(R, "pos"), &r->pos, r->tab_ntemp, npn);
}

static void cfg_from_struct(const mxArray *s, mpcekf_config *c) {
  mpcekf_config_defaults(c);
  if (!s || mxIsEmpty(s)) return;
  if (!mxIsStruct(s)) mexErrMsgIdAndTxt("mpcekf:arg", "cfg: expected a struct");
#define GETI(f) if (mxGetField(s, 0, #f)) c->f = (int32_t)scalar(mxGetField(s, 0, #f), #f)
#define GETD(f) if (mxGetField(s, 0, #f)) c->f = scalar(mxGetField(s, 0, #f), #f)
  GETI(Np); GETI(Nc); GETD(target_soc); GETD(Crate); GETD(u_max); GETD(du_min); GETD(du_max); GETD(v_min);
  GETD(v_max); GETD(phise_min); GETD(z_max); GETD(z_tol); GETI(use_current); GETI(use_voltage); GETI(use_eta);
  GETI(max_hild); GETD(hild_tol); GETD(SigmaV); GETD(SigmaW); GETI(max_warn); GETI(flags); GETI(method);
#undef GETI
#undef GETD
  if (c->method != MPCEKF_METHOD_OB && c->method != MPCEKF_METHOD_MB)
    mexErrMsgIdAndTxt("mpcekf:arg", "cfg.method: %d (expected 0 = 'OB' or 1 = 'MB', initKF.m:44-49)", (int)c->method);
  const mxArray *sx = mxGetField(s, 0, "SigmaX0");
  if (sx) {
    const double *v = dvec(sx, 6, "SigmaX0 (diagonal, 6)");
    for (int i = 0; i < 6; ++i) c->SigmaX0[i] = v[i];
  }
}

static mxArray *dmat(size_t r, size_t c) { return mxCreateDoubleMatrix((mwSize)r, (mwSize)c, mxREAL); }
static mxArray *imat(size_t r, size_t c) { return mxCreateNumericMatrix((mwSize)r, (mwSize)c, mxINT32_CLASS, mxREAL); }

static const double *opt_vec(const mxArray *a, size_t n, const char *what) {
  return (!a || mxIsEmpty(a)) ? NULL : dvec(a, n, what);
}

/* Every command builds its outputs in plhs[0..MAXOUT); mexFunction hands MATLAB the
 * first max(nlhs, 1) of them (MATLAB's plhs has room for no more) and frees the rest. */
#define MAXOUT 8
static void need(int nrhs, int k, const char *usage) {
  if (nrhs < k) mexErrMsgIdAndTxt("mpcekf:arg", "usage: mpcekf_mex(%s)", usage);
}

static int g_nlhs = 1; /* the caller's nargout: 'ekf' copies Xind back only when it is asked for */
static void gateway(mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  char cmd[32];
  if (nrhs < 1 || mxGetString(prhs[0], cmd, sizeof cmd)) mexErrMsgIdAndTxt("mpcekf:arg", "first argument: command");
  if (!strcmp(cmd, "create")) {
    if (nrhs != 5) mexErrMsgIdAndTxt("mpcekf:arg", "create(R, cfg, device, ncells)");
    mpcekf_rom r;
    mpcekf_config c;
    rom_from_struct(prhs[1], &r);
    cfg_from_struct(prhs[2], &c);
    int free_slot = 0;
    for (int i = 0; i < MAXCTX; ++i) free_slot = free_slot || g_live[i] == NULL;
    if (!free_slot) mexErrMsgIdAndTxt("mpcekf:arg", "create: %d contexts are live; destroy one first", MAXCTX);
    mpcekf_ctx *h = NULL;
    chk(mpcekf_ctx_create(&r, &c, (int)scalar(prhs[3], "device"), (int64_t)scalar(prhs[4], "ncells"), &h));
    track(h, 1);
    mexAtExit(destroy_all);
    plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
    *(uint64_t *)mxGetData(plhs[0]) = (uint64_t)(uintptr_t)h;
    return; /* the row-major copies are mxMalloc'd: MATLAB frees them (the context copied the ROM) */
  }
  if (!strcmp(cmd, "hildreth")) {
    if (nrhs != 7) mexErrMsgIdAndTxt("mpcekf:arg", "hildreth(E, F, M, gamma, lambda0, maxIter)");
    const size_t Nc = mxGetM(prhs[1]), nC = mxGetM(prhs[3]);
    if (mxGetNumberOfDimensions(prhs[1]) != 2 || mxGetN(prhs[1]) != Nc)
      mexErrMsgIdAndTxt("mpcekf:arg", "hildreth: E must be Nc x Nc");
    if (mxGetNumberOfDimensions(prhs[3]) != 2 || mxGetN(prhs[3]) != Nc)
      mexErrMsgIdAndTxt("mpcekf:arg", "hildreth: M must be nC x Nc (Nc = %zu)", Nc);
    double *E = rowmajor(prhs[1], "E"), *M = rowmajor(prhs[3], "M");
    const double *F = dvec(prhs[2], Nc, "F"), *g = dvec(prhs[4], nC, "gamma");
    plhs[1] = dmat(nC, 1);
    memcpy(mxGetDoubles(plhs[1]), dvec(prhs[5], nC, "lambda0"), nC * sizeof(double));
    plhs[0] = dmat(Nc, 1);
    mxArray *ne = imat(1, 1);
    chk(mpcekf_hildreth(0, 1, (int32_t)Nc, (int32_t)nC, E, F, M, g, mxGetDoubles(plhs[1]),
                        (int32_t)scalar(prhs[6], "maxIter"), 1e-6, mxGetDoubles(plhs[0]), (int32_t *)mxGetData(ne)));
    plhs[2] = mxCreateDoubleScalar((double)*(int32_t *)mxGetData(ne));
    mxDestroyArray(ne);
    return;
  }
  if (!strcmp(cmd, "predmat")) {
    if (nrhs != 6) mexErrMsgIdAndTxt("mpcekf:arg", "predmat(a, C, D, Np, Nc)");
    const int Np = (int)scalar(prhs[4], "Np"), Nc = (int)scalar(prhs[5], "Nc");
    double *P = (double *)mxMalloc((size_t)Np * 7 * sizeof(double)), *G = (double *)mxMalloc((size_t)Np * Nc * sizeof(double));
    chk(mpcekf_predmat(0, 1, Np, Nc, dvec(prhs[1], 6, "a"), dvec(prhs[2], 6, "C"), dvec(prhs[3], 1, "D"), P, G));
    plhs[0] = dmat((size_t)Np, 7);
    plhs[1] = dmat((size_t)Np, (size_t)Nc);
    for (int i = 0; i < Np; ++i) { /* row-major -> column-major */
      for (int k = 0; k < 7; ++k) mxGetDoubles(plhs[0])[i + (size_t)Np * k] = P[i * 7 + k];
      for (int k = 0; k < Nc; ++k) mxGetDoubles(plhs[1])[i + (size_t)Np * k] = G[i * Nc + k];
    }
    return;
  }
  static const char *const with_handle[] = {"destroy", "init", "step", "plant", "ekf", "linearize", "mpc",
                                            "graph", "mpcdiag", "get_state", "set_state", "scalars", "linfields"};
  int known = 0;
  for (size_t i = 0; i < sizeof with_handle / sizeof *with_handle; ++i) known = known || !strcmp(cmd, with_handle[i]);
  if (!known) mexErrMsgIdAndTxt("mpcekf:arg", "unknown command %s", cmd);
  if (nrhs < 2) mexErrMsgIdAndTxt("mpcekf:arg", "%s: missing handle", cmd);
  mpcekf_ctx *h = handle(prhs[1]);
  int64_t n = 0;
  int32_t NM = 0, nz = 0, ncon = 0;
  chk(mpcekf_ctx_info(h, &n, &NM, &nz, &ncon));
  const size_t nc = (size_t)n, nzz = (size_t)nz + 2;
  if (!strcmp(cmd, "destroy")) {
    track(h, 0);
    chk(mpcekf_ctx_destroy(h));
  } else if (!strcmp(cmd, "init")) {
    need(nrhs, 4, "'init', h, soc0_pct, tc_degC");
    chk(mpcekf_init_cells(h, dvec(prhs[2], nc, "soc0"), dvec(prhs[3], nc, "tc")));
  } else if (!strcmp(cmd, "step")) {
    need(nrhs, 3, "'step', h, nsteps[, tc]");
    const double nsd = scalar(prhs[2], "nsteps");
    if (!(nsd >= 0 && nsd <= 2147483647.0) || nsd != (double)(int32_t)nsd)
      mexErrMsgIdAndTxt("mpcekf:arg", "nsteps: expected a non-negative integer");
    const int32_t ns = (int32_t)nsd;
    const double *tc = nrhs > 3 ? opt_vec(prhs[3], nc * (size_t)ns, "tc (ncells x nsteps)") : NULL;
    for (int i = 0; i < 4; ++i) plhs[i] = dmat(nc, (size_t)ns);
    plhs[4] = imat(nc, (size_t)ns);
    chk(mpcekf_step(h, ns, tc, mxGetDoubles(plhs[0]), mxGetDoubles(plhs[1]), mxGetDoubles(plhs[2]),
                    mxGetDoubles(plhs[3]), (int32_t *)mxGetData(plhs[4]), 0));
  } else if (!strcmp(cmd, "plant")) {
    need(nrhs, 3, "'plant', h, iapp[, tc]");
    plhs[0] = dmat(1, nc);
    chk(mpcekf_plant_step(h, dvec(prhs[2], nc, "iapp"), nrhs > 3 ? opt_vec(prhs[3], nc, "tc") : NULL,
                          mxGetDoubles(plhs[0])));
  } else if (!strcmp(cmd, "ekf")) {
    need(nrhs, 4, "'ekf', h, vk, ik[, tk]");
    /* [zk, zbk, xm, xg]: Xind crosses back only when asked for (nargout > 2); it stays on
       the device for 'linearize' with empty zk / xm / xg either way */
    const int want_x = g_nlhs > 2;
    plhs[0] = dmat(nzz, nc);
    plhs[1] = dmat(nzz, nc);
    plhs[2] = want_x ? imat(4, nc) : mxCreateDoubleMatrix(0, 0, mxREAL);
    plhs[3] = want_x ? dmat(4, nc) : mxCreateDoubleMatrix(0, 0, mxREAL);
    chk(mpcekf_ekf_step(h, dvec(prhs[2], nc, "vk"), dvec(prhs[3], nc, "ik"),
                        nrhs > 4 ? opt_vec(prhs[4], nc, "tk") : NULL, mxGetDoubles(plhs[0]), mxGetDoubles(plhs[1]),
                        want_x ? (int32_t *)mxGetData(plhs[2]) : NULL, want_x ? mxGetDoubles(plhs[3]) : NULL));
  } else if (!strcmp(cmd, "linearize")) {
    need(nrhs, 5, "'linearize', h, zk, xm, xg[, tk]");
    /* empty zk, xm, xg: the device copies of the last 'ekf'; the records stay on the device
       (plhs[0] empty) for 'mpc' / 'mpcdiag' with an empty lin and for 'linfields' */
    const double *tk = nrhs > 5 ? opt_vec(prhs[5], nc, "tk") : NULL;
    if (mxIsEmpty(prhs[2]) && mxIsEmpty(prhs[3]) && mxIsEmpty(prhs[4])) {
      plhs[0] = mxCreateDoubleMatrix(0, 0, mxREAL);
      chk(mpcekf_linearize(h, NULL, NULL, NULL, tk, NULL));
    } else {
      plhs[0] = dmat(MPCEKF_LIN_SIZE, nc);
      chk(mpcekf_linearize(h, dvec(prhs[2], nzz * nc, "zk"), ivec(prhs[3], 4 * nc, "xm (4 x ncells)"),
                           dvec(prhs[4], 4 * nc, "xg"), tk, mxGetDoubles(plhs[0])));
    }
  } else if (!strcmp(cmd, "mpc")) {
    need(nrhs, 4, "'mpc', h, lin, soc_k1");
    /* [uk, nexec, J_uncon, J_final, norm_DU, viol]: iterMPC.m's command and its
       mpcData.cost row (iterMPC.m:89-95), 1 x ncells each */
    for (int i = 0; i < 6; ++i) plhs[i] = (i == 1 || i == 5) ? imat(1, nc) : dmat(1, nc);
    chk(mpcekf_mpc_step_ex(h, opt_vec(prhs[2], MPCEKF_LIN_SIZE * nc, "lin"), dvec(prhs[3], nc, "soc_k1"),
                           mxGetDoubles(plhs[0]), (int32_t *)mxGetData(plhs[1]), mxGetDoubles(plhs[2]),
                           mxGetDoubles(plhs[3]), mxGetDoubles(plhs[4]), (int32_t *)mxGetData(plhs[5])));
  } else if (!strcmp(cmd, "graph")) {
    if (nrhs < 3) mexErrMsgIdAndTxt("mpcekf:arg", "graph: enable flag");
    chk(mpcekf_set_graph(h, (int32_t)(mxGetScalar(prhs[2]) != 0.0)));
  } else if (!strcmp(cmd, "mpcdiag")) {
    need(nrhs, 3, "'mpcdiag', h, lin[, uk_1]");
    plhs[0] = mxCreateDoubleMatrix(7, (mwSize)nc, mxCOMPLEX);  /* interleaved (re, im): [ncells][7][2] */
    plhs[1] = dmat(7, nc);
    chk(mpcekf_mpc_diag(h, opt_vec(prhs[2], MPCEKF_LIN_SIZE * nc, "lin"), nrhs > 3 ? opt_vec(prhs[3], nc, "uk_1") : NULL,
                        (double *)mxGetComplexDoubles(plhs[0]), mxGetDoubles(plhs[1])));
  } else if (!strcmp(cmd, "get_state") || !strcmp(cmd, "set_state")) {
    /* the model-blend EKF state (xhat, SigmaX 6 x 6) is part of an MB context's checkpoint */
    mpcekf_config cc;
    chk(mpcekf_ctx_config(h, &cc));
    const int nf = cc.method == MPCEKF_METHOD_MB ? 7 : 6;
    const char *f[] = {"bigX", "ekf", "scal", "lambda", "warn", "status", "mb"};
    const size_t rows[] = {(size_t)NM * 6, (size_t)NM * 20, MPCEKF_NSCAL, (size_t)ncon, 1, 1, MPCEKF_MB_SIZE};
    mpcekf_state st;
    memset(&st, 0, sizeof st);
    if (cmd[0] == 'g') {
      plhs[0] = mxCreateStructMatrix(1, 1, nf, f);
      mxArray *a[7];
      for (int i = 0; i < nf; ++i) {
        a[i] = (i == 4 || i == 5) ? imat(1, nc) : dmat(rows[i], nc);
        mxSetField(plhs[0], 0, f[i], a[i]);
      }
      st.bigX = mxGetDoubles(a[0]); st.ekf = mxGetDoubles(a[1]); st.scal = mxGetDoubles(a[2]);
      st.lambda = mxGetDoubles(a[3]); st.warn = (int32_t *)mxGetData(a[4]); st.status = (int32_t *)mxGetData(a[5]);
      if (nf == 7) st.mb = mxGetDoubles(a[6]);
      chk(mpcekf_get_state(h, &st));
    } else {
      if (nrhs < 3 || !mxIsStruct(prhs[2])) mexErrMsgIdAndTxt("mpcekf:arg", "set_state(h, st): st must be a struct");
      const mxArray *s = prhs[2];
      st.bigX = (double *)dvec(field(s, "bigX"), rows[0] * nc, "bigX");
      st.ekf = (double *)dvec(field(s, "ekf"), rows[1] * nc, "ekf");
      st.scal = (double *)dvec(field(s, "scal"), rows[2] * nc, "scal");
      st.lambda = (double *)dvec(field(s, "lambda"), rows[3] * nc, "lambda");
      st.warn = ivec(field(s, "warn"), nc, "warn");
      st.status = ivec(field(s, "status"), nc, "status");
      /* an MB checkpoint saved before st.mb existed restores without it (NULL keeps the
         context's blend state, as the C-ABI allows) */
      if (nf == 7 && mxGetField(s, 0, "mb")) st.mb = (double *)dvec(mxGetField(s, 0, "mb"), rows[6] * nc, "mb (MB context)");
      chk(mpcekf_set_state(h, &st));
    }
  } else if (!strcmp(cmd, "linfields")) {
    /* out = mpcekf_mex('linfields', h, idx[, set]): rows idx (1-based MPCEKF_LIN_* + 1) of
       the device-resident records of the last 'linearize' with empty zk, k x ncells; set
       (k x ncells) is written into them first */
    need(nrhs, 3, "'linfields', h, idx[, set]");
    const size_t k = mxGetNumberOfElements(prhs[2]);
    if (k < 1 || k > MPCEKF_LIN_SIZE) mexErrMsgIdAndTxt("mpcekf:arg", "linfields: 1..%d slot indices", MPCEKF_LIN_SIZE);
    const double *idx = dvec(prhs[2], k, "idx");
    int32_t slots[MPCEKF_LIN_SIZE];
    for (size_t j = 0; j < k; ++j) {
      if (!(idx[j] >= 1 && idx[j] <= MPCEKF_LIN_SIZE) || idx[j] != (double)(int)idx[j])
        mexErrMsgIdAndTxt("mpcekf:arg", "linfields: idx(%zu) = %g is not a slot 1..%d", j + 1, idx[j], MPCEKF_LIN_SIZE);
      slots[j] = (int32_t)idx[j] - 1;
    }
    plhs[0] = dmat(k, nc);
    chk(mpcekf_lin_fields(h, slots, (int32_t)k, nrhs > 3 ? opt_vec(prhs[3], k * nc, "set (k x ncells)") : NULL,
                          mxGetDoubles(plhs[0])));
  } else if (!strcmp(cmd, "scalars")) {
    need(nrhs, 3, "'scalars', h, idx");
    const size_t k = mxGetNumberOfElements(prhs[2]);
    if (k < 1 || k > MPCEKF_NSCAL) mexErrMsgIdAndTxt("mpcekf:arg", "scalars: 1..%d slot indices", MPCEKF_NSCAL);
    const double *idx = dvec(prhs[2], k, "idx");
    int32_t slots[MPCEKF_NSCAL];
    for (size_t j = 0; j < k; ++j) {
      if (!(idx[j] >= 1 && idx[j] <= MPCEKF_NSCAL) || idx[j] != (double)(int)idx[j])
        mexErrMsgIdAndTxt("mpcekf:arg", "scalars: idx(%zu) = %g is not a slot 1..%d", j + 1, idx[j], MPCEKF_NSCAL);
      slots[j] = (int32_t)idx[j] - 1;
    }
    plhs[0] = dmat(k, nc); /* k x ncells column-major = the library's [ncells][k] */
    plhs[1] = imat(1, nc);
    plhs[2] = imat(1, nc);
    chk(mpcekf_get_scalars(h, slots, (int32_t)k, mxGetDoubles(plhs[0]), (int32_t *)mxGetData(plhs[1]),
                           (int32_t *)mxGetData(plhs[2])));
  } else {
    mexErrMsgIdAndTxt("mpcekf:arg", "unknown command %s", cmd);
  }
}

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  mxArray *out[MAXOUT] = {0};
  g_nlhs = nlhs;
  gateway(out, nrhs, prhs);
  const int keep = nlhs < 1 ? 1 : nlhs;
  if (keep > MAXOUT) mexErrMsgIdAndTxt("mpcekf:arg", "too many outputs");
  for (int i = 0; i < MAXOUT; ++i) {
    if (i < keep) {
      if (i > 0 && !out[i]) mexErrMsgIdAndTxt("mpcekf:arg", "output %d is not defined for this command", i + 1);
      plhs[i] = out[i];
    } else if (out[i]) {
      mxDestroyArray(out[i]);
    }
  }
}
