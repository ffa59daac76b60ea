/*
 * mpcqp_closed_loop.h -- C ABI of the device-side closed-loop step that surrounds the QP solve
 * (part of libmpcqp.so).  These kernels replace, for a batch of independent chasers:
 *
 *   mpcqp_cl_configure  <- configureDynamicConstraints(...) + the l/u splice
 *                          reference src/simhelpers.py:11-140, src/trajectorySimulate.py:339-347
 *   mpcqp_cl_step       <- controller select (MPC / LQR failsafe / deadbeat), input-norm clip,
 *                          discrete linear CW plant (+ additive noise), perfect-state estimate,
 *                          range/bearing measurement, termination test
 *                          reference src/trajectorySimulate.py:285-337
 *   mpcqp_cl_noise      <- noiseVec = sigMat @ random.normal(0, 1, 4)
 *                          reference src/trajectorySimulate.py:268,351-356 (counter-based stream
 *                          per global chaser id instead of numpy's global generator)
 *   mpcqp_clc_period    <- one sample period of the continuous-time nonlinear loop: controller
 *                          select at the sample, RK45 plant sub-steps (scipy solve_ivp restated,
 *                          see mpcqp_estimation.h), measurement, termination test per sub-step
 *                          reference src/trajectorySimulateC.py:325-409
 *
 * Per-instance arrays are device pointers, row-major [instance][k].  Scenario constants are
 * host values copied into the handle at creation.  Planar model only: nx = 4, nu = 2, ny = 5,
 * ndi = 2 (the reference's model, src/trajectorySimulate.py:73-97).
 */
#ifndef MPCQP_CLOSED_LOOP_H
#define MPCQP_CLOSED_LOOP_H
#include <stdint.h>

#include "mpcqp_estimation.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t Nx, Nc, Nb, m, nnzA;
  double Ad[16], Bd[8];          /* row-major 4x4, 4x2 */
  double rp, rtol, xr[4];        /* platform radius, tolerance radius, reference state */
  int32_t inTrack, isReject, has_debris;
  double center[2], side, detect; /* debris box as given (un-swapped) */
  double verts[8];                /* debris vertices in configureDynamicConstraints' order
                                     (already turned on its side for in-track runs) */
  double umin[7], umax[7];        /* bounds of one (u, s) block */
  double Kpf[8], Kif[2];          /* failsafe LQR with integral action, 2x4 and 2x1 */
  double Ktot[8], Ki[2];          /* deadbeat debris avoidance, 2x4 and 2x1 */
  double Crefx[4], Crefy[4];
  const int32_t *pos_c1, *pos_c2, *pos_slope; /* host, Nx+1 each: CSC positions of the varying
                                                 A values (pos_slope NULL when no debris) */
} mpcqp_cl_scenario;

typedef struct mpcqp_cl mpcqp_cl;

int mpcqp_cl_create(const mpcqp_cl_scenario *sc, int32_t batch, void *stream, mpcqp_cl **out);
int mpcqp_cl_destroy(mpcqp_cl *cl);

/* From estimates xest [B*6] = [x, y, vx, vy, dx, dy] write the varying A values into Ax [B*nnzA]
 * (the constant values must already be there) and the varying bounds into l, u [B*m] (the
 * constant rows must already be there).  In-track runs swap xest[0] and xest[1] in place afterwards
 * (reference quirk, src/simhelpers.py:72). */
int mpcqp_cl_configure(mpcqp_cl *cl, double *xest, double *Ax, double *l, double *u);

/* One control step after a solve.  Inputs: status [B], x_sol [B*n] (u0 read at u0_offset),
 * noise [B*4] or NULL (noiseVec added to the plant update).
 * State in/out: x_true [B*4], ctrl_prev [B*2] (the control applied this step: one-sample delay,
 * src/trajectorySimulate.py:323-324), xintf [B], xest [B*6] (set to [x_true, 0, 0]), done [B]
 * (1 once the termination test fired; such instances are frozen), ctrl_seq [B] (1 MPC,
 * 2 failsafe, 3 deadbeat, 0 frozen; output), ctrl_out [B*2] (the control chosen this step).
 * Optional outputs (NULL to skip): z [B*2] the range/bearing measurement of the new true state,
 * u_applied [B*2] the control the plant applied (the UKF's predict input). */
int mpcqp_cl_step(mpcqp_cl *cl, const int32_t *status, const double *x_sol, int32_t n,
                  int32_t u0_offset, double *x_true, double *ctrl_prev, double *xintf,
                  double *xest, int32_t *done, int32_t *ctrl_seq, double *ctrl_out,
                  const double *noise, double *z, double *u_applied);

/* Per-chaser run summary kept up to date by every following mpcqp_cl_step (device buffers [B],
 * all four or none; NULL disables; the caller initialises them: iterm = nsim (or 0 for chasers
 * terminated at x0), success = 0, final_err = 0, n_fallback = 0):
 *   iterm      loop index at which the termination test fired (src/trajectorySimulate.py:288-293)
 *   success    1 once a state x(i), 1 <= i < iterm, is within dist_tol of xr with approach angle
 *              |atan(vy / vx)| <= ang_tol degrees (the reference's success test, :369-376)
 *   final_err  |x(iterm - 1) - xr|_2 (test/disturbRejComp.py:88), or of the last state stepped
 *   n_fallback steps that used the failsafe / deadbeat controller instead of the MPC solution
 * The step index counts mpcqp_cl_step calls on this handle. */
int mpcqp_cl_set_tracking(mpcqp_cl *cl, int32_t *iterm, int32_t *success, double *final_err,
                          int32_t *n_fallback, double dist_tol, double ang_tol);

/* Global id of instance 0 of this handle (a rank's shard offset); keys the noise streams. */
int mpcqp_cl_set_ids(mpcqp_cl *cl, int64_t id0);

/* noise [B*4] = [sig_x g0, sig_y g1, 0, 0], g ~ N(0, 1) from Philox-4x32-10 with key seed and
 * counter (draw, global id): draw k of chaser id is the same in every sharding. */
int mpcqp_cl_noise(mpcqp_cl *cl, uint64_t seed, uint64_t draw, double sig_x, double sig_y,
                   double *noise);

/* Continuous-time plant of mpcqp_clc_period (isDeltaV: the control is an impulse added to the
 * velocity at the sample instead of a held acceleration, src/trajectorySimulateC.py:375-380). */
int mpcqp_cl_set_plant(mpcqp_cl *cl, const mpcqp_plant_model *model, int32_t isDeltaV);

/* One sample period: loop iterations i_start .. i_start + nsub - 1 of trajectorySimulateC, the
 * first at a sample instant (a solve has just been enqueued).  Arguments as mpcqp_cl_step, plus
 * iterm [B] (set to the loop index at which the termination test fired), t_start (the
 * reference's `time` at i_start), dt = T_cont, and traj [B*nsub*4] or NULL (x after every
 * sub-step).  noise [B*4] is added after every sub-step; z / xest are taken after the first
 * sub-step, as the reference measures x(i_start + 1). */
int mpcqp_clc_period(mpcqp_cl *cl, const int32_t *status, const double *x_sol, int32_t n,
                     int32_t u0_offset, double *x_true, double *ctrl_prev, double *xintf,
                     double *xest, int32_t *done, int32_t *iterm, int32_t *ctrl_seq,
                     double *ctrl_out, const double *noise, double *z, double *u_applied,
                     double t_start, double dt, int32_t i_start, int32_t nsub, double *traj);

#ifdef __cplusplus
}
#endif
#endif
