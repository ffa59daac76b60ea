/*
 * mpcqp.h -- C ABI of libmpcqp.so, the MI355X-native batched MPC-QP engine.
 *
 * This is the drop-in boundary for the reference's hot path: the OSQP object that
 * src/trajectorySimulate.py / src/trajectorySimulateC.py create, set up and drive every control
 * step.  Each entry point replaces one OSQP call the reference makes (OSQP 0.6 C names in
 * brackets; the Python wrapper methods the reference calls are what a binding maps onto them):
 *
 *   mpcqp_create + mpcqp_set_data  <- osqp.OSQP(); prob.setup(P, q, A, l, u, warm_start=True,
 *                                     verbose=False)  [osqp_setup]
 *                                     reference src/trajectorySimulate.py:242-245,
 *                                               src/trajectorySimulateC.py:269-272
 *   mpcqp_update_bounds            <- prob.update(l=l, u=u)  [osqp_update_bounds]
 *                                     reference src/trajectorySimulate.py:342,
 *                                               src/trajectorySimulateC.py:399
 *   mpcqp_update_A (+ bounds)      <- prob.update(Ax=A.data, l=l, u=u)
 *                                     [osqp_update_bounds + osqp_update_A]
 *                                     reference src/trajectorySimulate.py:348,
 *                                               src/trajectorySimulateC.py:405
 *   mpcqp_solve                    <- res = prob.solve()  [osqp_solve]; the caller reads
 *                                     res.x[(Nx+1)*nx:(Nx+1)*nx+nu] and res.info.status
 *                                     reference src/trajectorySimulate.py:296-314,
 *                                               src/trajectorySimulateC.py:338-356
 *   mpcqp_warm_start               <- prob.warm_start(x=, y=)  [osqp_warm_start]
 *   mpcqp_destroy                  <- object destruction  [osqp_cleanup]
 *
 * Differences from OSQP by design: one handle holds a BATCH of B independent QPs that share the
 * sparsity pattern of P and A (and the values of P and q); A values and the bounds l, u are per
 * instance.  B = 1 is the reference's use.
 *
 * Rules
 *   - every function returns 0 on success and a negative MPCQP_E* code on failure; nothing throws
 *     across the ABI; mpcqp_last_error() gives a message for the calling thread;
 *   - structure arrays (mpcqp_structure) are HOST pointers read during mpcqp_create only;
 *   - every data pointer is a DEVICE pointer owned by the caller (e.g. a torch tensor's
 *     data_ptr()), laid out row-major [instance][element], float64 / int32;
 *   - work is enqueued on the HIP stream given to mpcqp_create and is asynchronous with respect to
 *     the host: synchronise the stream before reading outputs;
 *   - +-inf (or anything beyond +-1e30) in l/u means "no bound", as in OSQP;
 *   - a handle is not thread-safe.
 *   - status codes are OSQP 0.6's status_val (MPCQP_SOLVED == 1, ...), strings via
 *     mpcqp_status_string().
 */
#ifndef MPCQP_H
#define MPCQP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MPCQP_OK 0
#define MPCQP_E_INVALID (-1)      /* bad argument / dimension / pattern */
#define MPCQP_E_HIP (-2)          /* HIP runtime failure */
#define MPCQP_E_UNSUPPORTED (-3)  /* structure or setting this build cannot handle */
#define MPCQP_E_NODATA (-4)       /* solve before set_data */

/* linear-system engines (mpcqp_engine_kind) */
#define MPCQP_ENGINE_KKT 0    /* blocked level-scheduled LDL' of the quasi-definite KKT matrix */

/* OSQP 0.6 status_val values */
#define MPCQP_SOLVED 1
#define MPCQP_SOLVED_INACCURATE 2
#define MPCQP_PRIMAL_INFEASIBLE_INACCURATE 3
#define MPCQP_DUAL_INFEASIBLE_INACCURATE 4
#define MPCQP_MAX_ITER_REACHED (-2)
#define MPCQP_PRIMAL_INFEASIBLE (-3)
#define MPCQP_DUAL_INFEASIBLE (-4)
#define MPCQP_NON_CVX (-7)
#define MPCQP_UNSOLVED (-10)

typedef struct mpcqp_handle mpcqp_handle;

/* Shared sparsity: P upper-triangular CSC (n x n), A CSC (m x n), sorted row indices. */
typedef struct {
  int32_t n, m;
  const int32_t *Pp, *Pi; /* host, n+1 / nnz(P) */
  const int32_t *Ap, *Ai; /* host, n+1 / nnz(A) */
} mpcqp_structure;

/* OSQP 0.6 settings (same names, meaning and defaults; see mpcqp_default_settings). */
typedef struct {
  double rho, sigma, alpha;
  double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  double delta, adaptive_rho_tolerance;
  int32_t max_iter, scaling, adaptive_rho, adaptive_rho_interval;
  int32_t polish, polish_refine_iter, check_termination, warm_start, scaled_termination;
} mpcqp_settings;

/* Per-instance solve information written by mpcqp_solve (device pointers, may be NULL). */
typedef struct {
  int32_t *status;      /* [B] OSQP status_val */
  int32_t *iter;        /* [B] ADMM iterations */
  int32_t *rho_updates; /* [B] adaptive-rho refactorizations */
  double *obj_val;      /* [B] */
  double *pri_res;      /* [B] */
  double *dua_res;      /* [B] */
  double *rho;          /* [B] rho after the solve (carried into the next solve, as OSQP) */
} mpcqp_info;

int mpcqp_default_settings(mpcqp_settings *s);

/* Symbolic analysis (ordering, elimination tree, level schedules) + device allocation for a
 * batch of `batch` instances.  `stream` is a hipStream_t (NULL = default stream). */
int mpcqp_create(const mpcqp_structure *st, const mpcqp_settings *s, int32_t batch, void *stream,
                 mpcqp_handle **out);
int mpcqp_destroy(mpcqp_handle *h);

/* Problem data (device): Px [nnzP] and q [n] shared by all instances; Ax [B*nnzA] (CSC order),
 * l, u [B*m].  Resets the warm-start state of every instance (cold start, rho = settings.rho). */
int mpcqp_set_data(mpcqp_handle *h, const double *Px, const double *q, const double *Ax,
                   const double *l, const double *u);
/* New bounds for every instance [B*m] (device).  Alone (no mpcqp_update_A before the next solve)
 * this is osqp_update_bounds: the instance keeps its data scaling D, E, c -- the next solve re-runs
 * the Ruiz passes on the same unscaled data as the last scaling did, bitwise the same factors --
 * and the bounds are scaled by that E once. */
int mpcqp_update_bounds(mpcqp_handle *h, const double *l, const double *u);
/* New A values for every instance [B*nnzA] (device, CSC order): osqp_update_A.  The next solve of
 * each instance unscales its last scaled data (P, q, and the bounds as mpcqp_update_bounds scaled
 * them by the previous E), overwrites A and re-runs the Ruiz scaling -- OSQP 0.6's data drift. */
int mpcqp_update_A(mpcqp_handle *h, const double *Ax);
/* New shared linear cost q [n] (device). */
int mpcqp_update_lin_cost(mpcqp_handle *h, const double *q);
/* Warm start every instance from unscaled primal/dual guesses x [B*n], y [B*m] (device). */
int mpcqp_warm_start(mpcqp_handle *h, const double *x, const double *y);

/* Solve every instance (warm-started from its previous solve when settings.warm_start).
 * x [B*n], y [B*m] device outputs (unscaled, NaN when no solution exists, as OSQP). */
int mpcqp_solve(mpcqp_handle *h, double *x, double *y, const mpcqp_info *info);

/* Zero-copy access to the handle's own problem-data buffers (device): Ax [B*nnzA], l, u [B*m].
 * A producer kernel (e.g. mpcqp_cl_configure) may rewrite them in place between solves, on the
 * handle's stream.  Once Ax has been handed out, every later mpcqp_solve treats each instance as
 * updated by osqp_update_bounds + osqp_update_A (the reference's per-step pair,
 * src/trajectorySimulate.py:342,348); l / u alone do not change that. */
int mpcqp_data_buffers(mpcqp_handle *h, double **Ax, double **l, double **u);

/* Copy the current problem data of every instance into caller device buffers (any may be NULL):
 * Ax [B*nnzA], l, u [B*m]. */
int mpcqp_copy_data(mpcqp_handle *h, double *Ax, double *l, double *u);

/* Register a skip mask (device [B] int32, read by every following mpcqp_solve; NULL clears it):
 * instances with skip[i] != 0 are not solved and keep their outputs and warm state.  A batch of
 * closed loops passes its `done` flags, so chasers whose run has terminated cost nothing (the
 * reference stops calling solve() at termination, src/trajectorySimulate.py:288-296). */
int mpcqp_set_skip(mpcqp_handle *h, const int32_t *skip);
/* Solve order (device pointer, kept by the handle; NULL = instance order): a permutation of the B
 * instance ids, handed to the persistent waves in this order by the work counter.  Results are
 * unchanged (instances are independent); only the packing of the launch changes.  A closed loop
 * passes its chasers longest-first by the last solve's ADMM iterations, so the instances that run
 * to max_iter start first and the launch ends on short ones (no reference counterpart: OSQP solves
 * one problem at a time).  A non-permutation is undefined behaviour (a duplicate id races two
 * waves on one instance's warm state, a missing id is never solved); the array may be rewritten
 * between solves only on the handle's stream. */
int mpcqp_set_order(mpcqp_handle *h, const int32_t *order);

/* Copy the warm-start state the handle carries between solves (what OSQP keeps inside its
 * workspace) into caller device buffers (any may be NULL): the SCALED iterates xs [B*n], zs, ys
 * [B*m], rho [B] and has_state [B] (0: never solved / reset, 1: iterates of the last solve).
 * For white-box parity tests (the oracle's oqp_get_state counterpart). */
int mpcqp_get_state(const mpcqp_handle *h, double *xs, double *zs, double *ys, double *rho,
                    int32_t *has_state);
/* The reverse of mpcqp_get_state (device pointers, same layout): overwrite the warm-start state,
 * e.g. with another solver's iterates.  White-box parity tests only (the oracle's oqp_set_state
 * counterpart).  The data scaling is not part of this state: it stays the handle's own (an
 * instance this handle never solved scales its set-up data, whatever has_state says). */
int mpcqp_set_state(mpcqp_handle *h, const double *xs, const double *zs, const double *ys,
                    const double *rho, const int32_t *has_state);
/* The data scaling the handle carries between solves (caller device buffers, any may be NULL):
 * E [B*m], the row equilibration of the last solve (OSQP's scaling->E after its update_A), and the
 * unscaled P values Pu [B*nnzP] and q [B*n] that the next warm solve rescales -- OSQP 0.6's
 * unscale_data of the last scaled data, ((P_s c^-1) D^-1) D^-1 and (q_s c^-1) D^-1, so a warm
 * solve's Ruiz passes start from the same rounded data as osqp_update_A's.  White-box parity tests
 * (bitwise against the oracle's oqp_get_state / oqp_get_data). */
int mpcqp_get_scaling(const mpcqp_handle *h, double *E, double *Pu, double *qu);

/* Introspection. */
int mpcqp_dims(const mpcqp_handle *h, int32_t *n, int32_t *m, int32_t *nnzP, int32_t *nnzA,
               int32_t *nnzL);
/* Schedule statistics: number of level-scheduled steps of the factorization / forward / backward
 * triangular solves, LDS bytes per instance and resident waves (instances in flight) per CU. */
int mpcqp_schedule_info(const mpcqp_handle *h, int32_t *fac_steps, int32_t *fwd_steps,
                        int32_t *bwd_steps, int32_t *lds_bytes, int32_t *waves_per_cu);
/* Kind of the triangular-solve steps: *atomics_per_step = LDS atomic additions one lane issues per
 * solve step (3 for paired steps -- segments 0 + 1 of a lane summed into one target -- 4 otherwise).
 * The bench's LDS byte model reads it. */
int mpcqp_schedule_kind(const mpcqp_handle *h, int32_t *atomics_per_step);
/* The solve kernel the handle launches (any pointer may be NULL): *waves_per_instance (1, or 2 for
 * the two-wave kernel), *instances_per_cu (resident instances per CU: LDS image and registers),
 * *regs (registers per lane the kernel allocates, arch VGPRs + AGPRs, from hipFuncGetAttributes) and
 * *scratch_bytes (per-lane scratch).  mpcqp_create refuses a kernel above the validated register /
 * scratch budget (MPCQP_MAX_KERNEL_REGS / MPCQP_MAX_KERNEL_SCRATCH, DESIGN.md High-register builds). */
#define MPCQP_MAX_KERNEL_REGS 440
#define MPCQP_MAX_KERNEL_SCRATCH 512
int mpcqp_kernel_info(const mpcqp_handle *h, int32_t *waves_per_instance, int32_t *instances_per_cu,
                      int32_t *regs, int32_t *scratch_bytes);
/* Which linear-system engine the handle runs (MPCQP_ENGINE_KKT: the only engine of this build;
 * round 1's dense-inverse alternative measured slower and was removed). */
int mpcqp_engine_kind(const mpcqp_handle *h, int32_t *kind);
/* Host-only symbolic analysis (no HIP call; usable without a GPU): KKT ordering, L pattern and
 * schedule statistics for a structure.  perm [n+m], Lp [n+m+1] may be NULL; Li is written only
 * when non-NULL and *nnzL (in) >= the true count.  stats (may be NULL) receives
 * {fac_steps, fwd_steps, bwd_steps, fwd_levels, bwd_levels, lds_image_bytes}. */
int mpcqp_analyze(const mpcqp_structure *st, int32_t *perm, int32_t *Lp, int32_t *Li,
                  int32_t *nnzL, int32_t *stats);
/* Host-only schedule self-check (no HIP call): compiles the same plan mpcqp_create would and
 * interprets it on the CPU for one instance -- KKT assembly from Px (upper CSC of P), Ax (CSC of A),
 * sigma and rho_vec [m], the factorization schedule, then one forward / diagonal / backward solve
 * of [[P + sigma I, A'], [A, -diag(1/rho_vec)]] sol = rhs (sol, rhs [n+m], host arrays).  model
 * [4] (may be NULL) receives the modelled LDS cycles of one ADMM iteration's solve work for one
 * wave: solve-step reads, solve-step atomics, vector passes, and the conflict-free floor of the
 * same instructions.  Diagnostics / tests only; the product path never calls it. */
int mpcqp_schedule_check(const mpcqp_structure *st, const double *Px, const double *Ax,
                         double sigma, const double *rho_vec, const double *rhs, double *sol,
                         int64_t *model);

/* The same program as a KKT solver with the factorization and the solves apart (host-only,
 * diagnostics): mpcqp_emu_factor assembles [[P + sigma I, A'], [A, -diag(1/rho)]] from the
 * scaled values and runs the factorization schedule; mpcqp_emu_solve runs one forward /
 * diagonal / backward solve on it, rhs and sol [n + m] in the original order.  Bitwise the
 * device kernel's factorization and solves (tests/test_gpu_hybrid.py); the oracle's hybrid runs
 * use it in place of QDLDL. */
typedef struct mpcqp_emu mpcqp_emu;
int mpcqp_emu_create(const mpcqp_structure *st, mpcqp_emu **out);
/* another solver state on the same compiled program (shared, read-only) */
int mpcqp_emu_clone(const mpcqp_emu *src, mpcqp_emu **out);
int mpcqp_emu_destroy(mpcqp_emu *e);
int mpcqp_emu_factor(mpcqp_emu *e, const double *Px, const double *Ax, double sigma,
                     const double *rho_vec);
int mpcqp_emu_solve(mpcqp_emu *e, const double *rhs, double *sol);
/* Host-side export of the symbolic analysis for white-box tests (no device work):
 * perm [n+m] (KKT position -> original KKT index), Lp [n+m+1], Li [nnzL]. */
int mpcqp_export_symbolic(const mpcqp_handle *h, int32_t *perm, int32_t *Lp, int32_t *Li);
const char *mpcqp_status_string(int32_t status);
const char *mpcqp_last_error(void);
/* ABI version (major*100 + minor). */
int mpcqp_version(void);

#ifdef __cplusplus
}
#endif
#endif
