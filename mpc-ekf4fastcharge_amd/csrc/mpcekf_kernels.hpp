// mpcekf_kernels.hpp -- shared declarations between the C-ABI host code and the
// gfx950 kernels (mpcekf_kernels.hip).  Plain structs passed by value as kernel
// arguments; every pointer is a device pointer.
#pragma once
#include <cstddef>
#include <cstdint>

namespace mk {

constexpr int NX = 5;      // transient states per local model (initKF.m:60)
constexpr int NPK = 15;    // packed upper-triangular 5x5 covariance
constexpr int NA = 7;      // x_aug = [x(6); u] (predMat.m:20-22)
constexpr int REC = 20;    // per-model EKF record: xhat[5] + SigmaX packed[15]
constexpr int MAXT = 8;    // max temperature set-points
constexpr int MAXZ = 40;   // max SOC set-points
constexpr int MAXROWS = 64;
constexpr int NPLANT = 9;  // role rows the plant needs (OB_step.m:289-344)
constexpr int PREC = NPLANT * NX + NPLANT + NPLANT + 6;  // plant blob record per model: C[9][5], res0[9], D[9], a[6]
// 64: with the ring inputs of a replay loaded 8 steps per round trip (mpcekf_kernels.hip
// ring_chunk), the longer replays of a 64-step ring cost less than the halved flush saves
// (same-box A/B, profiles/r04f_ab_lazy64.txt: 2.64e8 vs 2.60e8); at 32 steps with a load per
// replayed step it had been the other way round
#ifndef MPCEKF_LAZY_H
#define MPCEKF_LAZY_H 64
#endif
constexpr int LAZY_H = MPCEKF_LAZY_H;  // deferred time update: input ring length = flush period (steps)
constexpr int MAXTT = 8;
constexpr int MBREC = 42;   // model-blend state per cell: xhat[5], pad, Sigma 6x6 row-major
constexpr int KF_MB = 1 << 8;  // KCfg.flags: model-blend EKF (mpcekf_config.method == 1)    // max electrode-table temperatures (mpcekf_rom.tab_ntemp)

// role slots = the first rows of the permuted output vector (rom.py ROLE_NAMES)
enum { R_IFDL0 = 0, R_IFDL3, R_IF0, R_IF3, R_TH0, R_TH3, R_TE1, R_TEE, R_PHIE, R_PHISE0, R_NPHISE2, NROLE };
// per-row group flags (rom.py G_*)
enum : unsigned { G_NTH = 1, G_PTH = 2, G_NPHISE = 4, G_PPHISE = 8, G_PHIE = 16, G_PHIE0 = 32, G_THETAE = 64,
                  G_PPHIS = 128 };
enum { C0_ZERO = 0, C0_CHATV0, C0_RES0N, C0_RES0P, C0_DUN, C0_DUP, C0_MDUN };
enum { ST_ERROR = 1, ST_LOCKOUT = 2, ST_THETAE_NEG = 4 };

struct KRom {
  int NM, nT, nZ, nz, nzp;  // nzp = padded row count the kernel was built for
  int nth, nte;                   // electrode tables: theta points, temperatures
  double Ts, Q, F, R, Rc, Tref;
  double th0n, th100n, th0p, th100p;  // theta0(), theta100() of the plant (OB_step.m:207-210)
  unsigned char flags[MAXROWS];   // per permuted row
  // the same flags as one row mask per flag bit (bit q: permuted row q carries flag 1 << b):
  // a kernel tests row q's flag with one scalar bit test on a mask (rowf), so the unrolled
  // row loops keep 8 uniform words live instead of a byte per row (rows >= 32 never reach
  // a kernel: nzp is 26 or 32)
  unsigned fmask[8];
  unsigned char c0k[MAXROWS];     // getChatZ Chat0 kind per permuted row
  short perm[MAXROWS];            // permuted row -> ROM row
  // blobs end with: electrode tables (mpcekf_kernels.hip ETab; *_tablen doubles), Tpts
  // [MAXT] (K), Zpts [MAXZ] (fraction)
  const double *cell_blob;        // per model [C nzp*5][D nzp][a 5] ... then tables
  int cell_stride, cell_tab, cell_tablen, cell_len;
  const double *plant_blob;       // per model [C 9*5][res0 9][D 9] ... then tables
  int plant_tab, plant_tablen, plant_len;
  const double *bulk_tab;         // cA[NM*20], cB[NM*20], cP[NM*6]
  // 1: the model rows of both blobs do not fit the 160 KiB LDS (large NM); the kernels
  // stage only the tables (from *_tab, even offsets) and read the model rows from HBM/L2
  int rom_global;
  // 1: the cell blob also carries the plant's res0 column per model (after the Sigma
  // coefficients) and the Cdleff tables, and the fused step runs OB_step's simStep at the
  // start of k_cell (no k_plant launch)
  int cell_plant;
  // ABI v3 electrode tables (mpcekf_kernels.hip ETab): npoly = KPOLY when the rows are
  // theta polynomials in `poly` (global, L2-resident), 0 for the v2 linear tables in LDS;
  // arr = any function has an Arrhenius factor.  Each function's rows and Ea/R are found
  // through its descriptor in the blobs' LDS table header (etab_desc, KDESC doubles each).
  // nodes = some function is on its own theta nodes (ABI v4: its descriptor names a bucket
  // map; the lookups test this uniform flag before reading it).
  int npoly, arr, nodes;
  const double *poly;
};
constexpr int KPOLY = 6;  // coefficients per theta interval the kernels evaluate (quintic; cubics padded)
constexpr int KDESC = 4;  // doubles per v3 / v4 lookup descriptor (mpcekf_kernels.hip etab_desc)
constexpr int KMAP = 4;   // doubles per v4 bucket-map entry: k0, x_k0, x_k0+1, 0

struct KCfg {
  double SigmaV, SigmaW, ref, u_max, u_min, du_min, du_max, v_max, phise_min, zmax, hild_tol;
  int max_warn, max_hild, flags;
};

struct KState {
  int64_t n;
  double *bigx;   // [n][NM][6]
  double *ekf;    // [n][NM][20]
  double *SOCn, *SOCp, *x0, *S0, *priorI, *uk_1, *uk, *vk;  // [n]
  double *lam;    // [ncon][n]
  int *warn, *status;
  // per-cell constants (set at init)
  double *Tc;  // the cell's temperature (degC): set at init, by per-call arguments and per fused step
  const double *SOC0, *SOC0n, *SOC0p;
  // diagnostics of the last MPC step
  double *J_unc, *J_fin;
  int *nviol;
  // hand-off k_cell -> k_hild
  int *hflag;      // [n] 1: hildreth.m must run this step (2: k_hild_slow finishes it)
  int *hslow;      // [1] waves of the current step with a k_hild_slow lane (k_plant zeroes it)
  double *prob;    // [PB_N][n] problem records (mpcekf_kernels.hip PB_*)
  double *mb;      // [n][MBREC] model-blend EKF state (method 'MB' only)
  // deferred all-model time update (fused mpcekf_step only): each local
  // model's record is current through step ts[c][m] of the running call; the inputs
  // of the last LAZY_H steps sit in per-cell rings
  int *ts_ekf, *ts_plant;    // [n][NM]
  double *hist_p, *hist_u;   // [LAZY_H][n] priorI (EKF) and Iapp (plant) of step t at slot t % LAZY_H
  long long *stamps;         // [NSTAMPS][n] section clocks (-DMPCEKF_STAMPS builds only, else null)
};

// Inputs/outputs of one cell-kernel launch.  Any pointer may be null.
struct KIO {
  int mode;               // MODE_* bits
  int64_t step_stride;    // unused (reserved)
  // fused trajectories, already offset to this step ([ncells])
  double *u, *v, *soc, *phise;
  int *nexec;
  double *zk, *zbk;       // [n][nz+2] (un-permuted)
  // stage entry points
  const double *vk_in, *ik_in;          // ekf stage
  int *xm_out; double *xg_out;          // [n][4]
  const double *zk_in; const int *xm_in; const double *xg_in;  // linearize stage
  double *lin_out; const double *lin_in;                        // [n][35]
  const double *soc_k1_in; double *uk_out;                      // mpc stage
  int lazy_t;             // > 0: fused step t of the running call with deferred time update
  double *bnd;            // [NBND][n] boundzk hand-off k_cell -> k_bounds (with zbk)
  long long *stamps;      // [MPCEKF_NSTAMPS][n] s_memtime per k_cell section (-DMPCEKF_STAMPS builds only)
  double *zsoc_out;       // [n] zk(end) for the wide-horizon MPC kernels (P_LIN, fused)
  // per-step diagnostics of the fused step (runMPC.m:106-111, mpcData.cost iterMPC.m:89-95)
  double *x_out;          // [n][6] x_store: the EKFmatsHandler xhat
  double *junc_out, *jfin_out, *normdu_out;  // [n] J_uncon, J_final, norm_DU
  int *nviol_out;         // [n] viol
  // fused step with KRom::cell_plant: OB_step's simStep runs first in k_cell (no k_plant);
  // tc_in (device [n] degC, may be null) is the step's TC, stored into s.Tc
  int plant;
  const double *tc_in;
  int hild;  // fused step, Np = 5: hildreth.m at the end of k_cell (no k_hild launch)
};
constexpr int NSTAMPS = 20;  // k_cell sections 0..11, k_plant 12..19
// k_cell -> k_bounds record: g[4], m[4], getChatZ's getChatV scalars at the updated state
// (Rfn, Rfp, Rctn, Rctp, dUn0, dUp3 of chat_k; its Chat0), res0n, res0p, dUn, dUp
// (iterEKF.m:562-580), SigmaX0.  k_bounds reads corner 1's Sigma from the EKF record
// k_cell stored (nothing writes it before the next k_cell).
enum { BD_G = 0, BD_M = 4, BD_K = 8, BD_C0 = 14, BD_R0N, BD_R0P, BD_DUN, BD_DUP, BD_S0, NBND };

enum { MODE_EKF = 1, MODE_LIN = 2, MODE_MPC = 4, MODE_FUSED = 8 };
// Which blocks of k_cell an instantiation compiles: the fused step launches the iterEKF
// part and the EKFmatsHandler + iterMPC part as two kernels (each with its own register
// allocation), handing over zk and Xind through HBM; the stage entry points use both.
enum { P_EKF = 1, P_MPC = 2, P_ALL = 3, P_LIN = 4 };  // P_EKF | P_LIN: iterEKF + EKFmatsHandler only (wide MPC)

// Scratch of the wide-horizon MPC stage (mpcekf_wide.hip; Np = 20, Nc = 10): the
// Hildreth problem, X = E\M', K = M*(E\F) + gamma and H_ii per constraint row.
struct KWide {
  int Np, Nc, ncon;
  double *prob;    // [wide_prob_doubles][n]: E, F, Hv, He, Hs, gamma, e, Ru, uk_1
  double *X;       // [ncon][n][Nc]  X(:,i) = E\M(i,:)' (the exact path's; k_hild_wide forms its own)
  double *R;       // [Nc(Nc+1)/2][n] chol(E) upper triangle by rows (k_hild_prep -> k_hild_wide)
  double *K, *hii; // [ncon][n]
  int *it;         // [n] hildreth.m sweeps (nexec)
  int *q;          // [1] fast-path cells this step (k_hild_sort)
  int *list;       // [n] those cells, longest predicted sweep count first (k_hild_bin)
  int *hist;       // [2 * 64] k_hild_bin's histogram of last step's counts | list offsets
  double *smin;    // [Nc*Nc + 1] GsocT*Gsoc of the configuration and its sigma_min
};

// host-side launchers (defined in mpcekf_kernels.hip)
// lazy_t > 0: deferred mode (corners replayed/advanced in place, inputs logged to the rings)
// tc_in (device, [n] degC, may be null): the step's temperature, stored into s.Tc first
int launch_plant(const KRom &r, const KState &s, const double *iapp, double *vout, int lazy_t, const double *tc_in,
                 void *stream);
// brings every model of every cell from its ts to step t, then sets ts = new_ts
// every model of cells [c_lo, c_hi) (c_hi < 0: to the end) brought to step t, timestamps new_ts
int launch_flush(const KRom &r, const KCfg &c, const KState &s, int t, int new_ts, void *stream, int64_t c_lo = 0,
                 int64_t c_hi = -1);
int launch_bulk(const KRom &r, const KCfg &c, const KState &s, const double *iapp, int do_plant, int do_ekf,
                void *stream);
int launch_cell(const KRom &r, const KCfg &c, const KState &s, const KIO &io, void *stream, int parts = P_ALL);
// the fused step's iterEKF ('OB') with a lane quad per cell (nT > 1 and nZ > 1): zk /
// Xind hand-off in io.zk / io.xm_out / io.xg_out for k_cell<P_MPC>, boundzk record in io.bnd
int launch_ekf4(const KRom &r, const KCfg &c, const KState &s, const KIO &io, void *stream, int block = 512);
// boundzk (iterEKF.m:186-205) from k_cell's hand-off record, a lane quad per cell
int launch_bounds(const KRom &r, const KState &s, const double *bnd, double *zbk, void *stream);
int launch_hild(const KCfg &c, const KState &s, const KIO &io, void *stream);
constexpr int PROB_DOUBLES = 51;  // PB_N for Np = 5, Nc = 2
int launch_predmat(int64_t n, int Np, int Nc, const double *a, const double *C, const double *D, double *Phi,
                   double *G, void *stream);
int launch_constraints(const KCfg &c, int64_t n, const double *lin, const double *uk_1, const double *soc_k1,
                       double *M, double *gam, void *stream);
// (Nc, ncon) = (2, 23): the compiled form; any other Nc <= 10, ncon <= 100: the runtime-sized
// form, which needs hildreth_any_scratch(n, Nc, ncon) doubles of device scratch
int launch_hildreth(int64_t n, int Nc, int ncon, const double *E, const double *F, const double *M,
                    const double *gam, double *lam, int max_iter, double tol, double *DU, int *nexec,
                    void *stream, double *scratch);
size_t hildreth_any_scratch(int64_t n, int Nc, int ncon);
int launch_hildreth_structured(int64_t n, const double *E, const double *F, const double *Hv, const double *He,
                               const double *Hs, const double *gam, double *lam, int max_iter, double tol,
                               double *DU, int *nexec, void *stream);
int launch_init_state(int64_t n, int NM, double *ekf, double *bigx, const double *sx0, void *stream);
bool cell_kernel_supported(int nzp);
bool cell_computes_bounds();  // k_cell evaluates boundzk itself (no k_bounds launch, no hand-off record)
bool cell_runs_hild();        // the fused step's k_cell also runs hildreth.m when KIO::hild is set

// wide-horizon MPC stage (mpcekf_wide.hip)
bool wide_supported(int Np, int Nc);
int wide_prob_doubles(int Np, int Nc);
// GsocT*Gsoc + sigma_min cache for mpc_setup (rr = -Ts/(3600 Q), a = diag(A) of one model)
int launch_wide_smin(const KWide &w, double rr, const double *a6, void *stream);
// iterMPC setup from the linearisation records io.lin_in [n][35] and io.soc_k1_in [n]
int launch_mpc_wide(const KCfg &c, const KState &s, const KIO &io, const KWide &w, void *stream);
// iterMPC.m:53-60 poles / sv from this step's linearisation records and pre-step uk_1
// (Np = 5 / Nc = 2 here, the wide horizons in mpcekf_wide.hip)
int launch_cl_diag(const KCfg &c, int64_t n, const double *lin, const double *uk1, double *poles, double *sv,
                   void *stream);
int launch_cl_diag_wide(const KCfg &c, int64_t n, const double *lin, const double *uk1, double *poles, double *sv,
                        void *stream);
// hildreth.m (16-lane groups, exact lane-per-cell path for the rest) and iterMPC.m:75-95
int launch_hild_wide(const KCfg &c, const KState &s, const KIO &io, const KWide &w, void *stream);
// context-free predMat / constraintsMPC / hildreth at the wide horizons
int launch_predmat_wide(int64_t n, int Np, int Nc, const double *a, const double *C, const double *D, double *Phi,
                        double *G, void *stream);
int launch_constraints_wide(const KCfg &c, int Np, int Nc, int64_t n, const double *lin, const double *uk_1,
                            const double *soc_k1, double *M, double *gam, void *stream);
// selected columns of [n][stride] records to / from a compact [n][k] buffer (mpcekf_io.hip)
int launch_cols(double *rec, int64_t n, int stride, const int *slots, int k, double *compact, bool scatter,
                void *stream);
int cell_lds_bytes(const KRom &r);
int bounds_lds_bytes(const KRom &r, int block);
int plant_lds_bytes(const KRom &r);

}  // namespace mk
