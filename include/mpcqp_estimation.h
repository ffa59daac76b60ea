/*
 * mpcqp_estimation.h -- C ABI of the device-side state estimator and nonlinear plant that surround
 * the QP solve in the reference's closed loops (part of libmpcqp.so).  Batched: B independent
 * chasers, per-instance arrays are device pointers, row-major [instance][k]; calls are
 * asynchronous on the handle's stream; int return codes (0 ok, -1 invalid argument, -2 HIP error).
 *
 *   mpcqp_ukf_step    <- filterpy UnscentedKalmanFilter(dim_x=6, dim_z=2, fx, hx,
 *                        MerweScaledSigmaPoints(6, alpha, beta, kappa)): kf.predict(u) then
 *                        kf.update(z)  (filterpy 1.4.5, not installed here; restated)
 *                        reference src/trajectorySimulate.py:113-130,271-282,329-337
 *                                  src/trajectorySimulateC.py:140-157,310-320,384-392
 *                        fx(x, u) = Ao x + Bou u,  hx(x) = [|x[0:2]|, atan2(x[1], x[0])]
 *   mpcqp_plant_rk45  <- per sub-step: soln = scipy.integrate.solve_ivp(stateEqnN,
 *                        (t, t + T_cont), x, args=(u,)); x = soln.y[:, -1] + w; t = t + T_cont
 *                        reference src/trajectorySimulateC.py:64-79,371-380,409 (scipy 1.15.3 RK45)
 */
#ifndef MPCQP_ESTIMATION_H
#define MPCQP_ESTIMATION_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- unscented Kalman filter */
typedef struct {
  double Ao[36], Bou[12]; /* fx(x, u) = Ao x + Bou u (row-major 6x6, 6x2) */
  double Q[36], R[4];     /* kf.Q, kf.R */
  double alpha, beta, kappa; /* MerweScaledSigmaPoints parameters */
} mpcqp_ukf_model;

typedef struct mpcqp_ukf mpcqp_ukf;

int mpcqp_ukf_create(const mpcqp_ukf_model *model, int32_t batch, void *stream, mpcqp_ukf **out);
int mpcqp_ukf_destroy(mpcqp_ukf *ukf);

/* One kf.predict(u) + kf.update(z) per instance.  x [B*6] and P [B*36] (kf.x, kf.P) in/out;
 * u [B*2], z [B*2].  active [B] or NULL: instances with active[b] == 0 are left untouched.
 * status [B] out: 0 ok; 1 the Cholesky factorisation of (lambda + n) P failed (filterpy raises
 * LinAlgError there) -- x and P are then set to NaN. */
int mpcqp_ukf_step(mpcqp_ukf *ukf, double *x, double *P, const double *u, const double *z,
                   const int32_t *active, int32_t *status);

/* ------------------------------------------------------------ nonlinear plant (RK45) */
typedef struct {
  /* the Python-float constants of stateEqnN, evaluated as the reference does:
   * two_n = 2*n, m_two_n = -2*n, n2 = n**2, R_T = 500e3 + 6378.1e3, mu = n**2 * R_T**3,
   * g0 = mu / R_T**2 */
  double two_n, m_two_n, n2, R_T, mu, g0;
  double rtol, atol; /* solve_ivp tolerances (reference: defaults 1e-3, 1e-6) */
} mpcqp_plant_model;

/* nsub consecutive sub-steps from time t0 with step dt, for every instance:
 *   x <- solve_ivp(stateEqnN, (t, t + dt), x, args=(u,)).y[:, -1] + w ;  t <- t + dt
 * x [B*4] in/out; u [B*2] held over the sub-steps (the acceleration input; pass zeros for the
 * delta-v model); w [B*4] or NULL (additive state noise per sub-step); traj [B*nsub*4] or NULL
 * (the state after every sub-step); failed [B] or NULL (set to 1 where the integrator reported a
 * step-size failure, solve_ivp status -1). */
int mpcqp_plant_rk45(const mpcqp_plant_model *model, int32_t batch, void *stream, double *x,
                     const double *u, const double *w, double t0, double dt, int32_t nsub,
                     double *traj, int32_t *failed);

#ifdef __cplusplus
}
#endif
#endif
