/*
 * mpcekf.h -- C-ABI of the MI355X batched MPC+EKF fast-charge control step.
 *
 * Drop-in boundary for the per-timestep loop of Rodrigops27/MPC-EKF4FastCharge
 * (runMPC.m:83-112).  The reference has no FFI of its own: its public surface
 * is the set of MATLAB functions runMPC.m calls by name.  Each entry point below
 * replaces one of them, batched over independent cells:
 *
 *   mpcekf_plant_step   <- [Vcell,obs,cellState] = OB_step(Iapp,Tc,cellState,ROM)  OB_step.m:1
 *   mpcekf_ekf_step     <- [zk,boundzk,ekfData,Xind] = iterEKF(vk,ik,Tk,ekfData)    iterEKF.m:30
 *   mpcekf_linearize    <- [MPC,xhat] = EKFmatsHandler(ekfData,Xind,zk,Tk)         EKFmatsHandler.m:1
 *   mpcekf_predmat      <- [Phi,G,aug] = predMat(A,B,C,D,Np,Nc)                    predMat.m:1
 *   mpcekf_constraints  <- [M,gamma] = constraintsMPC(x_aug_k,cellState,mpcData)   constraintsMPC.m:1
 *   mpcekf_mpc_step     <- [uk,mpcData] = iterMPC(xk,cellState,mpcData)            iterMPC.m:1
 *   mpcekf_hildreth     <- [DU,lambda,nexec] = hildreth(E,F,M,gamma,lambda0,maxIter) hildreth.m:1
 *   mpcekf_init_cells   <- initKF.m:30, initMPC.m:29, first OB_step call (runMPC.m:20,52,74)
 *   mpcekf_step         <- the fused loop body runMPC.m:84-111, nsteps times
 *   mpcekf_step_ex      <- the same, with every runMPC.m store (zkEst, zkBound, x_store,
 *                          mpcData.cost) per step
 *
 * Conventions
 *  - Plain C types only; no exceptions cross the ABI.  Every function returns an
 *    int status (MPCEKF_OK == 0); on failure mpcekf_last_error() returns a
 *    thread-local message.
 *  - Batched arrays are cell-major ("[ncells][k]") unless stated; trajectories
 *    are step-major "[nsteps][ncells]".  All floating point is IEEE fp64.
 *  - Host pointers unless the argument is documented as "device".  Every call
 *    synchronises its HIP stream before returning.
 *  - Per-cell soft failures never fail a call: they set bits in the per-cell
 *    status word (MPCEKF_ST_*), after which that cell's outputs are NaN.  This
 *    replaces the MATLAB errors/NaN lock-out of iterEKF.m:55-59,384-389.
 *  - One context = one GPU + one HIP stream; use one host thread per context.
 *    Multi-GPU runs create one context per device on disjoint cell ranges.
 */
#ifndef MPCEKF_H
#define MPCEKF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCEKF_ABI_VERSION 4

/* return codes */
#define MPCEKF_OK 0
#define MPCEKF_E_ARG -1         /* bad argument / size                                  */
#define MPCEKF_E_ROM -2         /* ROM fails the initKF/iterEKF/OB_step structure checks */
#define MPCEKF_E_HIP -3         /* HIP runtime error                                     */
#define MPCEKF_E_UNSUPPORTED -4 /* configuration not built into this library             */
#define MPCEKF_E_STATE -5       /* call order (e.g. step before init_cells)              */

/* per-cell status bits */
#define MPCEKF_ST_ERROR 1      /* cell stopped; outputs NaN from here on                       */
#define MPCEKF_ST_LOCKOUT 2    /* warnCount > max_warn at iterEKF entry (iterEKF.m:55-59)      */
#define MPCEKF_ST_THETAE_NEG 4 /* thetae < 0 in getVariables; MATLAB errors (iterEKF.m:384-389) */

/* tfData.names codes (tf_code[] of mpcekf_rom) */
enum {
  MPCEKF_TF_negIfdl = 0, MPCEKF_TF_posIfdl, MPCEKF_TF_negIf, MPCEKF_TF_posIf, MPCEKF_TF_negIdl,
  MPCEKF_TF_posIdl, MPCEKF_TF_negPhis, MPCEKF_TF_posPhis, MPCEKF_TF_negPhise, MPCEKF_TF_posPhise,
  MPCEKF_TF_negThetass, MPCEKF_TF_posThetass, MPCEKF_TF_negPhie, MPCEKF_TF_sepPhie,
  MPCEKF_TF_posPhie, MPCEKF_TF_negThetae, MPCEKF_TF_sepThetae, MPCEKF_TF_posThetae,
  MPCEKF_TF_COUNT
};

/* One electrode's cellData.function.{neg,pos} handles in tabulated form.
 * The 2-D tables are [ntemp][ntheta] (row j = the handle at T = rom.tab_T_K[j] over a
 * uniform theta grid on [0, 1]) and are evaluated by the defined bilinear interpolation
 * (theta clamped to [0, 1], T clamped to the grid ends; ntemp == 1: theta only).
 * ABI v3 (rom.tab_npoly = 4 or 6): each row is instead a piecewise polynomial in theta,
 * *_p [ntemp][ntheta-1][tab_npoly] (Uocp1_p [ntheta-1][tab_npoly]): on interval i of the
 * grid, with s = theta (ntheta-1) - i in [0, 1], c0 + s (c1 + s (... + s c_last)) (the
 * exporter fits Hermite cubics / quintics to the handles' values and theta-derivatives);
 * the node tables above stay required (the v2 route and the checks read them).  Ea[f]
 * != 0 multiplies function f (EF order Uocp, dUocp, k0, Rf, Cdleff), after the T
 * interpolation, by its Arrhenius factor exp(Ea/R (1/Tref - 1/T)) with the call's T
 * (unclamped); its rows then hold f / that factor.  So a handle k(th)exp(Ea/R(1/Tref - 1/T))
 * is exact in T, an OCP U0(th) + (T - Tref) dUdT(th) is exact in T between table rows:
 *   soc(z,T)     = soc0(T) + z*(soc100(T) - soc0(T))   iterEKF.m:282-283,439-440,497-498;
 *                                                      EKFmatsHandler.m:57-58; OB_step.m:64-65
 *   Uocp(th,T)   = Uocp       OB_step.m:313-314,337-338; iterEKF.m:362-363,404-405; EKFmatsHandler.m:84-85
 *   Uocp(th)     = Uocp1      the one-argument call, EKFmatsHandler.m:96
 *   dUocp(th,T)  = dUocp      OB_step.m:231-232; iterEKF.m:495-496,579-580
 *   k0(th,T)     = k0         OB_step.m:329-330; iterEKF.m:392-393,463-464; EKFmatsHandler.m:60-61
 *   Rf(th,T)     = Rf         OB_step.m:339-340; iterEKF.m:406-407,441-442; EKFmatsHandler.m:68-69
 *   Cdl(th,T)^(2-nDL) * wDL(th,T)^(nDL-1) = Cdleff, read at th = SOC0n/p (OB_step.m:212-219)
 * theta0/theta100 are the zero-argument calls the plant makes (OB_step.m:207-210). */
typedef struct {
  double theta0, theta100;
  const double *soc0, *soc100;                 /* [ntemp] soc(0,T), soc(1,T)       */
  const double *Uocp, *dUocp, *k0, *Rf, *Cdleff; /* [ntemp][ntheta] each            */
  const double *Uocp1;                         /* [ntheta]                         */
  /* ABI v3: theta polynomials of the same functions (NULL when tab_npoly == 0) */
  const double *Uocp_p, *dUocp_p, *k0_p, *Rf_p, *Cdleff_p; /* [ntemp][ntheta-1][tab_npoly] */
  const double *Uocp1_p;                                   /* [ntheta-1][tab_npoly]        */
  double Ea[5];            /* J/mol: Arrhenius factor of Uocp, dUocp, k0, Rf, Cdleff; 0 = none */
  /* ABI v4 (tab_npoly != 0): a function on its own theta nodes -- a lookup-table handle
   * (interp1 / pchip over measured breakpoints, which no uniform-grid polynomial follows
   * across a slope break).  Index f: Uocp, dUocp, k0, Rf, Cdleff, Uocp1.  nnode[f] = 0: the
   * uniform-grid *_p above; m = nnode[f] >= 2: node[f] [m] strictly ascending (interior nodes
   * in (0, 1)) and node_p[f] [ntemp][m-1][tab_npoly] (Uocp1: [m-1][tab_npoly]), segment k's
   * polynomial in d = theta - node[f][k]: theta clamped to [0, 1], k = #{j in 1..m-2 :
   * node[f][j] <= theta} (the end segments extend past the end nodes), then Horner and the
   * temperature blend and Arrhenius factor as for v3.  The uniform *_p of such a function may
   * be NULL.  An interp1-linear row is (y_k, slope_k, 0, 0): the handle's value to rounding. */
  int32_t nnode[6];
  const double *node[6];
  const double *node_p[6];
} mpcekf_electrode;

/* The ROM struct of runMPC.m:5 as plain arrays.  Set-points ascending. */
typedef struct {
  int32_t nT, nZ;          /* ROMmdls is nT x nZ                                  */
  int32_t n;               /* transient states per model (must be 5)               */
  int32_t nz;              /* outputs per model                                    */
  const double *T_degC;    /* xraData.T   [nT]                                     */
  const double *SOC_pct;   /* xraData.SOC [nZ]                                     */
  double Ts;               /* xraData.Tsamp                                        */
  const double *A;         /* [nT][nZ][n+1]      diag(ROMmdls(t,z).A), last == 1   */
  const double *C;         /* [nT][nZ][nz][n+1]  ROMmdls(t,z).C (with res0 column) */
  const double *D;         /* [nT][nZ][nz]       ROMmdls(t,z).D                    */
  const int32_t *tf_code;  /* [nz] MPCEKF_TF_*   tfData.names                      */
  const double *tf_xloc;   /* [nz]               tfData.xLoc                       */
  double F, R, Q, Rc, Tref;
  int32_t tab_ntheta;      /* theta grid points of the electrode tables (>= 2)     */
  int32_t tab_ntemp;       /* temperature grid points (>= 1)                       */
  const double *tab_T_K;   /* [tab_ntemp] ascending, Kelvin                        */
  int32_t tab_npoly;       /* ABI v3: 0 = linear tables; 4 / 6 = cubic / quintic *_p (and v4 node_p) */
  mpcekf_electrode neg, pos;
} mpcekf_rom;

#define MPCEKF_CF_BOUNDS 1 /* also compute boundzk (iterEKF.m:186-205) */

/* Controller/estimator configuration (runMPC.m:8-50, initMPC.m). */
typedef struct {
  int32_t Np, Nc;          /* horizons (runMPC.m:28-29)                          */
  double target_soc;       /* mpcData.ref, percent (runMPC.m:30)                 */
  double Crate;            /* u_min = -Q*Crate (initMPC.m:66-67)                 */
  double u_max, du_min, du_max, v_min, v_max, phise_min, z_max, z_tol;
  int32_t use_current, use_voltage, use_eta; /* constraint switches (runMPC.m:33) */
  int32_t max_hild;        /* mpcData.maxHild (initMPC.m:47)                     */
  double hild_tol;         /* hildreth.m:39 (1e-6)                               */
  double SigmaV, SigmaW;   /* runMPC.m:18-19                                     */
  double SigmaX0[6];       /* diagonal of SigmaX0 (runMPC.m:17)                  */
  int32_t max_warn;        /* lock-out threshold (iterEKF.m:55: > 10)            */
  int32_t flags;           /* MPCEKF_CF_*                                        */
  int32_t method;          /* initKF.m:44-49 blend: MPCEKF_METHOD_OB (runMPC.m) or _MB */
} mpcekf_config;

#define MPCEKF_METHOD_OB 0 /* output blend: every local model filtered (iterEKF.m 'OB')      */
#define MPCEKF_METHOD_MB 1 /* model blend: one blended model per cell (iterEKF.m:90-102 'MB') */

/* Layout of one linearisation record (EKFmatsHandler outputs), doubles: */
#define MPCEKF_LIN_A 0     /* [6] diag(A)              */
#define MPCEKF_LIN_CSOC 6  /* [6] Csoc                 */
#define MPCEKF_LIN_DSOC 12 /* Dsoc                     */
#define MPCEKF_LIN_CV 13   /* [6] [Cv 0]               */
#define MPCEKF_LIN_DV 19   /* Dv                       */
#define MPCEKF_LIN_CPHI 20 /* [6] [Cphi 0]             */
#define MPCEKF_LIN_DPHI 26 /* Dphi                     */
#define MPCEKF_LIN_BV 27   /* bv                       */
#define MPCEKF_LIN_BPHI 28 /* bphi                     */
#define MPCEKF_LIN_XHAT 29 /* [6] xhat (model + 0)     */
#define MPCEKF_LIN_SIZE 35

typedef struct mpcekf_ctx mpcekf_ctx;

int mpcekf_abi_version(void);
/* sha256 prefix of the sources this library was built from (profiles record the one
 * they were measured on; bench.py refuses stale PMC figures). */
const char *mpcekf_build_id(void);
const char *mpcekf_last_error(void);
void mpcekf_config_defaults(mpcekf_config *cfg); /* the runMPC.m values */

/* Context: owns the device copy of the ROM and the per-cell state (SoA/AoS in HBM). */
int mpcekf_ctx_create(const mpcekf_rom *rom, const mpcekf_config *cfg, int device, int64_t ncells,
                      mpcekf_ctx **out);
int mpcekf_ctx_destroy(mpcekf_ctx *ctx);
int mpcekf_ctx_info(const mpcekf_ctx *ctx, int64_t *ncells, int32_t *nmodels, int32_t *nz, int32_t *ncon);
/* The configuration the context was created with (e.g. its method, for a checkpoint). */
int mpcekf_ctx_config(const mpcekf_ctx *ctx, mpcekf_config *cfg);

/* initKF + initMPC + OB_step first call for every cell: SOC0 in percent, Tc in degC
 * (the cell temperature until a call passes another one). */
int mpcekf_init_cells(mpcekf_ctx *ctx, const double *soc0_pct, const double *tc_degC);

/* nsteps fused closed-loop steps.  tc_degC is the temperature runMPC.m:85-92 passes to
 * OB_step, iterEKF and EKFmatsHandler at each step, [nsteps][ncells] in degC, or NULL to
 * keep every cell's current temperature.  Each output may be NULL; non-NULL outputs are
 * [nsteps][ncells] host arrays (or device arrays when outputs_on_device != 0, which
 * then also applies to tc_degC):
 *   traj_u = u_store (MPC command), traj_v = voltage_store, traj_soc = SOC_store
 *   (zk(end)), traj_phise = phise_store, traj_nexec = mpcData.cost.nexec. */
int mpcekf_step(mpcekf_ctx *ctx, int32_t nsteps, const double *tc_degC, double *traj_u, double *traj_v,
                double *traj_soc, double *traj_phise, int32_t *traj_nexec, int32_t outputs_on_device);

/* Per-step outputs of mpcekf_step_ex (runMPC.m:55-69 stores, filled at runMPC.m:94-111
 * and iterMPC.m:89-95).  Every pointer may be NULL.  Step-major arrays, host pointers
 * (device pointers when outputs_on_device != 0):
 *   [nsteps][ncells]       u, v, soc, phise, nexec, J_unc, J_fin, norm_du, nviol
 *   [nsteps][ncells][6]    x    (x_store: the EKFmatsHandler xhat, integrator state last)
 *   [nsteps][ncells][nz+2] zk, zbk (zkEst / zkBound; zbk needs MPCEKF_CF_BOUNDS)
 *   [nsteps][ncells][7][2] poles (mpcData.poles = eig(CL), iterMPC.m:53-59: re, im;
 *                          sorted by descending real, then imaginary part)
 *   [nsteps][ncells][7]    sv    (mpcData.sv = svd(CL), iterMPC.m:60, descending)
 * A cell in error has NaN floating outputs and zero nexec / nviol from its failing step on. */
typedef struct {
  double *u, *v, *soc, *phise;     /* u_store, voltage_store, SOC_store, phise_store    */
  int32_t *nexec;                  /* mpcData.cost.nexec                                */
  double *x;                       /* x_store                                           */
  double *zk, *zbk;                /* zkEst, zkBound                                    */
  double *J_unc, *J_fin, *norm_du; /* mpcData.cost.J_uncon / J_final / norm_DU          */
  int32_t *nviol;                  /* mpcData.cost.viol                                 */
  double *poles, *sv;              /* mpcData.poles, mpcData.sv (stability diagnostics) */
} mpcekf_traj;
int mpcekf_step_ex(mpcekf_ctx *ctx, int32_t nsteps, const double *tc_degC, const mpcekf_traj *traj,
                   int32_t outputs_on_device);

/* Optional per-step EKF output of the LAST mpcekf_step call: zk and boundzk
 * ([ncells][nz+2], boundzk only with MPCEKF_CF_BOUNDS). */
int mpcekf_get_zk(mpcekf_ctx *ctx, double *zk, double *boundzk);

/* eig / svd of one n x n (n <= 8) row-major matrix on the host, as the fused step
 * computes mpcData.poles / mpcData.sv (iterMPC.m:57-60): re/im sorted by descending real
 * then imaginary part, sv descending; any output may be NULL.  Returns MPCEKF_E_ARG for
 * n outside 1..8; non-finite input gives NaN outputs. */
int mpcekf_cl_eig(int32_t n, const double *a, double *re, double *im, double *sv);

/* ---- stage entry points (one MATLAB function each; all batched over cells) ----
 * Each has an _async twin with the same arguments ("every call returns
 * after hipStreamSynchronize unless _async is used"): it enqueues the call's copies and
 * kernels on the context's stream in order and returns without waiting.  Host inputs are
 * copied before it returns (the caller may free or reuse them; an input above
 * MPCEKF_BOUNCE_MAX bytes is read in place and must stay alive until the synchronisation).
 * Host outputs are written by the time mpcekf_sync(ctx) or the next synchronous stage call
 * returns -- not before; the caller keeps those arrays alive and unread until then.  Errors
 * of the enqueued copies are reported by that synchronisation.  The synchronous calls copy
 * outputs in chunks whose DMA overlaps the host-side copy (a worker pool, MPCEKF_CHUNK bytes
 * per chunk, MPCEKF_COPY_THREADS workers).
 * The temperature argument (Tc of OB_step.m:1, Tk of iterEKF.m:30 / EKFmatsHandler.m:1,
 * degC, [ncells]) sets each cell's temperature for this and later calls; NULL keeps it. */
/* OB_step: applies iapp[c] to the plant state at tc_degC[c], returns vcell[c] (may be NULL:
 * Vcell also stays on the device for the next mpcekf_ekf_step with vk = NULL). */
int mpcekf_plant_step(mpcekf_ctx *ctx, const double *iapp, const double *tc_degC, double *vcell);
/* iterEKF: zk/boundzk [ncells][nz+2], xind_model [ncells][4] (model index t*nZ+z of
 * Xind.theT/theZ), xind_gamma [ncells][4].  Every output may be NULL: zk and Xind also stay
 * on the device for the next mpcekf_linearize (runMPC.m:91 -> :94 without a host round trip).
 * vk = NULL: the last mpcekf_plant_step's Vcell on the device (MPCEKF_E_STATE without one). */
int mpcekf_ekf_step(mpcekf_ctx *ctx, const double *vk, const double *ik, const double *tk_degC, double *zk,
                    double *boundzk, int32_t *xind_model, double *xind_gamma);
/* EKFmatsHandler: lin [ncells][MPCEKF_LIN_SIZE], or NULL (the record stays on the device for
 * mpcekf_mpc_step / mpcekf_mpc_diag with lin = NULL and mpcekf_lin_fields).  zk, xind_model and
 * xind_gamma are all given, or all NULL for the device copies of the last mpcekf_ekf_step
 * (MPCEKF_E_STATE if there was none since init / the last fused step / set_state). */
int mpcekf_linearize(mpcekf_ctx *ctx, const double *zk, const int32_t *xind_model, const double *xind_gamma,
                     const double *tk_degC, double *lin);
/* Selected slots (MPCEKF_LIN_*) of the device-resident linearisation records of the last
 * mpcekf_linearize: out [ncells][nslots] (may be NULL), and set [ncells][nslots] (may be NULL)
 * written into those slots first -- e.g. runMPC.m:95-96 reads MPC.Cphi / Dphi / bphi and xhat
 * (14 doubles of the 35), and an iterMPC caller with another xk writes MPCEKF_LIN_XHAT.. */
int mpcekf_lin_fields(mpcekf_ctx *ctx, const int32_t *slots, int32_t nslots, const double *set, double *out);
/* iterMPC (uses and updates the context's uk_1 and lambda warm start):
 * soc_k1 = mpcData.SOCk_1 per cell; outputs uk, nexec.  lin = NULL: the device-resident
 * record of the last mpcekf_linearize; soc_k1 = NULL: zk(end) of the last mpcekf_ekf_step on
 * the device (runMPC.m:99's mpcData.SOCk_1 = zk(end)). */
int mpcekf_mpc_step(mpcekf_ctx *ctx, const double *lin, const double *soc_k1, double *uk, int32_t *nexec);
/* The same, also returning this call's iterMPC.m:89-95 cost log (mpcData.cost.J_uncon,
 * J_final, norm_DU, viol) per cell; any of the four may be NULL. */
int mpcekf_mpc_step_ex(mpcekf_ctx *ctx, const double *lin, const double *soc_k1, double *uk, int32_t *nexec,
                       double *J_unc, double *J_fin, double *norm_du, int32_t *nviol);
/* iterMPC.m:53-60 stability analysis of the iterMPC that mpcekf_mpc_step would run on lin:
 * Kmpc = first row of E\(G_soc'*Phi_soc), CL = Abar - Bbar*Kmpc; poles [ncells][7][2]
 * (eig(CL): re, im, sorted as in mpcekf_traj), sv [ncells][7] (svd(CL)).  uk_1 [ncells]
 * (mpcData.uk_1) or NULL for the context's current one (call before mpcekf_mpc_step).
 * Reads nothing else of the context's state and changes none of it.  lin = NULL: the
 * device-resident record of the last mpcekf_linearize. */
int mpcekf_mpc_diag(mpcekf_ctx *ctx, const double *lin, const double *uk_1, double *poles, double *sv);
/* the _async twins (see above) */
int mpcekf_plant_step_async(mpcekf_ctx *ctx, const double *iapp, const double *tc_degC, double *vcell);
int mpcekf_ekf_step_async(mpcekf_ctx *ctx, const double *vk, const double *ik, const double *tk_degC, double *zk,
                          double *boundzk, int32_t *xind_model, double *xind_gamma);
int mpcekf_linearize_async(mpcekf_ctx *ctx, const double *zk, const int32_t *xind_model, const double *xind_gamma,
                           const double *tk_degC, double *lin);
int mpcekf_lin_fields_async(mpcekf_ctx *ctx, const int32_t *slots, int32_t nslots, const double *set, double *out);
int mpcekf_mpc_step_async(mpcekf_ctx *ctx, const double *lin, const double *soc_k1, double *uk, int32_t *nexec);
int mpcekf_mpc_step_ex_async(mpcekf_ctx *ctx, const double *lin, const double *soc_k1, double *uk, int32_t *nexec,
                             double *J_unc, double *J_fin, double *norm_du, int32_t *nviol);
int mpcekf_mpc_diag_async(mpcekf_ctx *ctx, const double *lin, const double *uk_1, double *poles, double *sv);

/* Context-free batched kernels (device chosen by `device`).
 * predMat with A = diag(a), B = ones: a,C [n][6], D [n] -> Phi [n][Np][7], G [n][Np][Nc]. */
int mpcekf_predmat(int device, int64_t n, int32_t Np, int32_t Nc, const double *a, const double *C,
                   const double *D, double *Phi, double *G);
/* constraintsMPC: lin [n][LIN], uk_1/soc_k1 [n] -> M [n][ncon][Nc], gamma [n][ncon]. */
int mpcekf_constraints(int device, const mpcekf_config *cfg, double Q, int64_t n, const double *lin,
                       const double *uk_1, const double *soc_k1, double *M, double *gamma);
/* hildreth: E [n][Nc][Nc], F [n][Nc], M [n][ncon][Nc], gamma/lambda [n][ncon]; lambda is
 * the warm start in and the multipliers out; DU [n][Nc]; nexec [n].  Any M with
 * 1 <= Nc <= 10 and 1 <= ncon <= 100 (hildreth.m:1; Nc = 2 / ncon = 23 is the compiled
 * fused-path form, other sizes a runtime-sized kernel with the same defined arithmetic). */
int mpcekf_hildreth(int device, int64_t n, int32_t Nc, int32_t ncon, const double *E, const double *F,
                    const double *M, const double *gamma, double *lambda, int32_t max_iter, double tol,
                    double *DU, int32_t *nexec);

/* hildreth.m for the constraint pattern of constraintsMPC.m as runMPC configures it
 * (Np = 5, Nc = 2, all three switches): M = [Cu; -Cu; I; -I; G_v; -G_e; G_soc] given by
 * the Toeplitz columns Hv, He, Hs [n][5] (G_v(i,j) = Hv(i-j) for j <= i).  This is the
 * solver the fused step runs (rank-2 form, hildreth.m:17-46); E [n][2][2], F [n][2],
 * gamma/lambda [n][23], DU [n][2], nexec [n] as in mpcekf_hildreth. */
int mpcekf_hildreth_structured(int device, int64_t n, const double *E, const double *F, const double *Hv,
                               const double *He, const double *Hs, const double *gamma, double *lambda,
                               int32_t max_iter, double tol, double *DU, int32_t *nexec);

/* ---- instrumentation (not part of the reference interface) ---- */
/* When enabled, mpcekf_step brackets every kernel launch with HIP events on the
 * context's stream; enable = N > 1 samples steps N-1, 2N-1, ... and the last only (the
 * events then perturb the timed stream N times less; with N dividing 32 the sampled steps
 * include every flush).  mpcekf_get_timing returns the summed milliseconds and launch
 * counts of [plant, flush, cell, hild, bounds] (arrays of MPCEKF_NKERNELS) since the
 * last call and resets them.  "flush" is the all-model time update (k_flush, every
 * 32 steps and at the end of each call); "bounds" is boundzk (k_bounds, when
 * MPCEKF_CF_BOUNDS is set). */
#define MPCEKF_K_PLANT 0
#define MPCEKF_K_FLUSH 1
#define MPCEKF_K_CELL 2
#define MPCEKF_K_HILD 3
#define MPCEKF_K_BOUNDS 4
#define MPCEKF_NKERNELS 5
int mpcekf_set_timing(mpcekf_ctx *ctx, int32_t enable);
/* Graph replay of the fused call (runMPC.m:83-112's loop as a device graph, SURVEY.md
 * §8(f) row 2): with enable != 0, mpcekf_step / mpcekf_step_ex capture each new call
 * shape (nsteps, output and temperature buffers, diagnostics) into a hipGraph once and
 * replay it on later calls of the same shape -- the per-step launches of a control loop
 * that calls mpcekf_step(ctx, 1, ...) every period become one graph launch.  Results are
 * identical; ignored while mpcekf_set_timing is on.  Also MPCEKF_GRAPH=1 at create. */
int mpcekf_set_graph(mpcekf_ctx *ctx, int32_t enable);
int mpcekf_get_timing(mpcekf_ctx *ctx, double *ms_sum, int64_t *launches);
/* The Hildreth problem records of the last fused step, as k_cell left them for
 * k_hild (field-major [MPCEKF_PROB_DOUBLES][ncells]: E(2x2) F(2) Hv(5) He(5) Hs(5)
 * gamma(23) e(5) Ru uk_1), and hflag [ncells] (1 = the QP ran).  For replaying the
 * solver offline (tools/micro); either pointer may be NULL. */
#define MPCEKF_PROB_DOUBLES 51
int mpcekf_get_hild_problems(mpcekf_ctx *ctx, double *prob, int32_t *hflag);
/* Profiling builds only (-DMPCEKF_STAMPS, tools/stamps.py): shader-clock stamps at the
 * section boundaries of the EKF/MPC kernel (rows 0..11) and the plant kernel (rows
 * 12..19) for the last fused step, [MPCEKF_NSTAMPS][ncells].  Rows 12..19 are written
 * only when the plant runs as its own kernel (k_plant4: MPCEKF_CELL_PLANT=0 or the
 * lane-quad path); when it runs inside k_cell (the default) they read 0.  *nstamps = 0
 * (and nothing written) in normal builds.  ABI v3: 20 rows (v2 had 12). */
#define MPCEKF_NSTAMPS 20
int mpcekf_get_stamps(mpcekf_ctx *ctx, int64_t *stamps, int32_t *nstamps);

/* ---- device memory (not part of the reference interface) ----
 * Device buffers for outputs_on_device calls, allocated by the library's own HIP
 * runtime so a host process never holds a second one (a framework's bundled
 * runtime must not hand its pointers to these kernels).  mpcekf_dev_copy is
 * synchronous; kind is MPCEKF_COPY_*.  mpcekf_dev_copy2d copies `height` rows of
 * `width` bytes with the given pitches (e.g. every k-th cell of a [nsteps][ncells]
 * trajectory: width 8, spitch 8k).  mpcekf_sync waits for every launch of the
 * context's device. */
#define MPCEKF_COPY_H2D 0
#define MPCEKF_COPY_D2H 1
#define MPCEKF_COPY_D2D 2
int mpcekf_dev_alloc(int device, int64_t bytes, void **ptr);
int mpcekf_dev_free(void *ptr);
int mpcekf_dev_copy(void *dst, const void *src, int64_t bytes, int32_t kind);
int mpcekf_dev_copy2d(void *dst, int64_t dpitch, const void *src, int64_t spitch, int64_t width, int64_t height,
                      int32_t kind);
int mpcekf_sync(mpcekf_ctx *ctx);  /* also completes the _async stage calls' host outputs */

/* ---- state access (open-loop parity, checkpoint/restore) ---- */
typedef struct {
  double *bigX;    /* [ncells][NM][6]   OB_step cellState.bigX (column per model)     */
  double *ekf;     /* [ncells][NM][20]  per model: xhat[5], SigmaX packed upper [15] */
  double *scal;    /* [ncells][MPCEKF_NSCAL] scalars, see MPCEKF_S_*                 */
  double *lambda;  /* [ncells][ncon]    mpcData.lambda                               */
  int32_t *warn;   /* [ncells]          iterEKF warnCount                            */
  int32_t *status; /* [ncells]          MPCEKF_ST_*                                   */
  double *mb;      /* [ncells][MPCEKF_MB_SIZE] method MB: ekfData.xhat(1:5), 0, SigmaX
                      6x6 row-major (xhat(end) is MPCEKF_S_X0); may be NULL          */
} mpcekf_state;

#define MPCEKF_MB_SIZE 42

#define MPCEKF_S_SOCNAVG 0 /* cellState.SOCnAvg          */
#define MPCEKF_S_SOCPAVG 1 /* cellState.SOCpAvg          */
#define MPCEKF_S_X0 2      /* ekfData.x0                 */
#define MPCEKF_S_SIGMAX0 3 /* ekfData.SigmaX0            */
#define MPCEKF_S_PRIORI 4  /* ekfData.priorI             */
#define MPCEKF_S_UK_1 5    /* mpcData.uk_1               */
#define MPCEKF_S_UK 6      /* command applied next step  */
#define MPCEKF_S_VK 7      /* last plant voltage         */
#define MPCEKF_NSCAL 8

/* Every non-NULL field of st is copied; NULL fields are neither read nor written (a
 * checkpoint without mb restores an MB context's other fields and keeps its blend state). */
int mpcekf_get_state(mpcekf_ctx *ctx, mpcekf_state *st);
int mpcekf_set_state(mpcekf_ctx *ctx, const mpcekf_state *st);
/* The few per-cell scalars a stage-call host reads every step (the MATLAB drop-ins:
 * cellState.SOCnAvg/SOCpAvg before OB_step, OB_step.m:226-228; ekfData.x0, SigmaX0,
 * priorI, warnCount and the status after iterEKF): slots[nslots] are MPCEKF_S_* indices,
 * scal [ncells][nslots]; warn / status [ncells] may be NULL.  Only these bytes cross
 * PCIe: 8 * nslots (+ 4 + 4) per cell. */
int mpcekf_get_scalars(mpcekf_ctx *ctx, const int32_t *slots, int32_t nslots, double *scal, int32_t *warn,
                       int32_t *status);
int mpcekf_get_scalars_async(mpcekf_ctx *ctx, const int32_t *slots, int32_t nslots, double *scal, int32_t *warn,
                             int32_t *status);

#ifdef __cplusplus
}
#endif
#endif /* MPCEKF_H */
