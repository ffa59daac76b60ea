// plant_dev.hpp -- device code of the nonlinear relative-motion plant of trajectorySimulateC and of
// the integrator the reference runs it with.
//
// stateEqnN: reference src/trajectorySimulateC.py:64-79 (Hill frame, 500 km circular orbit, exact
// two-body gravity of a point mass at distance R_T + x, plus the commanded acceleration u).
//
// rk45_interval: scipy.integrate.solve_ivp(fun, (t0, t1), y0, args=(u,)) with the defaults the
// reference uses (method 'RK45', rtol 1e-3, atol 1e-6, max_step inf, no t_eval) returning y at t1
// (reference src/trajectorySimulateC.py:373,376 read soln.y[:, -1]).  Restated from scipy 1.15.3
// (the version in this image): scipy/integrate/_ivp/common.py select_initial_step / norm,
// rk.py rk_step / RungeKutta._step_impl / RK45 (Dormand-Prince 5(4) tableau), base.py
// OdeSolver.step, ivp.py solve_ivp's stepping loop.  Same step-size control, same accept/reject
// rule, same operation order where numpy's is defined; products and sums are explicitly rounded so
// the compiler cannot contract them into FMAs (accept/reject decisions then differ from scipy's
// only when an error norm lies within rounding of 1).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace mpcqp {

struct PlantConsts {
  // the reference's Python-float constants, evaluated on the host exactly as stateEqnN does:
  // two_n = 2 * n, m_two_n = -2 * n, n2 = n ** 2, R_T = 500e3 + 6378.1e3, mu = n**2 * R_T**3,
  // g0 = mu / R_T**2
  double two_n, m_two_n, n2, R_T, mu, g0;
  double rtol, atol;
};

__device__ __forceinline__ double pm(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double pa(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double ps(double a, double b) { return __dsub_rn(a, b); }

// dxdt of stateEqnN, left-to-right evaluation as in the Python expression
__device__ __forceinline__ void plant_rhs(const PlantConsts& c, const double y[4], double u0,
                                          double u1, double f[4]) {
  const double rx = pa(c.R_T, y[0]);
  const double den = pow(pa(pm(rx, rx), pm(y[1], y[1])), 1.5);
  f[0] = y[2];
  f[1] = y[3];
  f[2] = pa(pa(ps(pa(pm(c.two_n, y[3]), pm(c.n2, y[0])), __ddiv_rn(pm(c.mu, rx), den)), c.g0), u0);
  f[3] = pa(ps(pa(pm(c.m_two_n, y[2]), pm(c.n2, y[1])), __ddiv_rn(pm(c.mu, y[1]), den)), u1);
}

// RMS norm of v / s (common.norm: np.linalg.norm(x) / x.size ** 0.5, size 4)
__device__ __forceinline__ double rms4_div(const double v[4], const double s[4]) {
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double q = __ddiv_rn(v[i], s[i]);
    acc = pa(acc, pm(q, q));
  }
  return __ddiv_rn(sqrt(acc), 2.0);
}

// Dormand-Prince 5(4) (scipy RK45.C / A / B / E)
struct DP45 {
  static constexpr double C1 = 0.2, C2 = 0.3, C3 = 0.8, C4 = 8.0 / 9.0, C5 = 1.0;
  static constexpr double A10 = 0.2;
  static constexpr double A20 = 3.0 / 40.0, A21 = 9.0 / 40.0;
  static constexpr double A30 = 44.0 / 45.0, A31 = -56.0 / 15.0, A32 = 32.0 / 9.0;
  static constexpr double A40 = 19372.0 / 6561.0, A41 = -25360.0 / 2187.0, A42 = 64448.0 / 6561.0,
                          A43 = -212.0 / 729.0;
  static constexpr double A50 = 9017.0 / 3168.0, A51 = -355.0 / 33.0, A52 = 46732.0 / 5247.0,
                          A53 = 49.0 / 176.0, A54 = -5103.0 / 18656.0;
  static constexpr double B0 = 35.0 / 384.0, B1 = 0.0, B2 = 500.0 / 1113.0, B3 = 125.0 / 192.0,
                          B4 = -2187.0 / 6784.0, B5 = 11.0 / 84.0;
  static constexpr double E0 = -71.0 / 57600.0, E1 = 0.0, E2 = 71.0 / 16695.0, E3 = -71.0 / 1920.0,
                          E4 = 17253.0 / 339200.0, E5 = -22.0 / 525.0, E6 = 1.0 / 40.0;
};

// one rk_step: K[0] = f; stages 1..5; y_new; f_new = K[6]
__device__ __forceinline__ void rk_step(const PlantConsts& c, const double y[4], const double f[4],
                                        double h, double u0, double u1, double K[7][4],
                                        double ynew[4]) {
  using D = DP45;
  double yy[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) K[0][i] = f[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) yy[i] = pa(y[i], pm(pm(K[0][i], D::A10), h));
  plant_rhs(c, yy, u0, u1, K[1]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    yy[i] = pa(y[i], pm(pa(pm(K[0][i], D::A20), pm(K[1][i], D::A21)), h));
  plant_rhs(c, yy, u0, u1, K[2]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    yy[i] = pa(y[i], pm(pa(pa(pm(K[0][i], D::A30), pm(K[1][i], D::A31)), pm(K[2][i], D::A32)), h));
  plant_rhs(c, yy, u0, u1, K[3]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    yy[i] = pa(y[i], pm(pa(pa(pa(pm(K[0][i], D::A40), pm(K[1][i], D::A41)), pm(K[2][i], D::A42)),
                           pm(K[3][i], D::A43)),
                        h));
  plant_rhs(c, yy, u0, u1, K[4]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    yy[i] = pa(y[i],
               pm(pa(pa(pa(pa(pm(K[0][i], D::A50), pm(K[1][i], D::A51)), pm(K[2][i], D::A52)),
                        pm(K[3][i], D::A53)),
                     pm(K[4][i], D::A54)),
                  h));
  plant_rhs(c, yy, u0, u1, K[5]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    ynew[i] = pa(y[i], pm(h, pa(pa(pa(pa(pa(pm(K[0][i], D::B0), pm(K[1][i], D::B1)),
                                           pm(K[2][i], D::B2)),
                                        pm(K[3][i], D::B3)),
                                     pm(K[4][i], D::B4)),
                                  pm(K[5][i], D::B5))));
  plant_rhs(c, ynew, u0, u1, K[6]);
}

// solve_ivp(fun, (t0, t1), y, args=(u,)) -> y(t1); returns false if the solver failed (step size
// below 10 ulp of t: scipy status -1, y then holds the last accepted state)
__device__ inline bool rk45_interval(const PlantConsts& c, double t0, double t1, double y[4],
                                     double u0, double u1) {
  using D = DP45;
  const double rtol = c.rtol, atol = c.atol;
  double f[4];
  plant_rhs(c, y, u0, u1, f);
  // ---- select_initial_step (direction +1, error estimator order 4, max_step inf)
  const double interval = fabs(ps(t1, t0));
  if (interval == 0.0) return true;  // OdeSolver.step: t == t_bound -> finished, y unchanged
  double h_abs;
  {
    double sc[4], yv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sc[i] = pa(atol, pm(fabs(y[i]), rtol));
    const double d0 = rms4_div(y, sc);
    const double d1 = rms4_div(f, sc);
    double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : __ddiv_rn(pm(0.01, d0), d1);
    h0 = fmin(h0, interval);
#pragma unroll
    for (int i = 0; i < 4; ++i) yv[i] = pa(y[i], pm(pm(h0, 1.0), f[i]));
    double f1[4], df[4];
    plant_rhs(c, yv, u0, u1, f1);
#pragma unroll
    for (int i = 0; i < 4; ++i) df[i] = ps(f1[i], f[i]);
    const double d2 = __ddiv_rn(rms4_div(df, sc), h0);
    double h1;
    if (d1 <= 1e-15 && d2 <= 1e-15)
      h1 = fmax(1e-6, pm(h0, 1e-3));
    else
      h1 = pow(__ddiv_rn(0.01, fmax(d1, d2)), 0.2);
    h_abs = fmin(fmin(pm(100.0, h0), h1), interval);
  }
  // ---- stepping loop (solve_ivp / OdeSolver.step / RungeKutta._step_impl)
  double t = t0;
  for (;;) {
    if (t == t1) return true;
    const double min_step = pm(10.0, fabs(ps(nextafter(t, __builtin_inf()), t)));
    if (h_abs < min_step) h_abs = min_step;
    bool rejected = false;
    double K[7][4], ynew[4], t_new;
    for (;;) {
      if (h_abs < min_step) return false;
      t_new = pa(t, h_abs);
      if (ps(t_new, t1) > 0) t_new = t1;
      const double h = ps(t_new, t);
      h_abs = fabs(h);
      rk_step(c, y, f, h, u0, u1, K, ynew);
      double sc[4], err[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sc[i] = pa(atol, pm(fmax(fabs(y[i]), fabs(ynew[i])), rtol));
        const double e = pa(pa(pa(pa(pa(pa(pm(K[0][i], D::E0), pm(K[1][i], D::E1)),
                                          pm(K[2][i], D::E2)),
                                       pm(K[3][i], D::E3)),
                                    pm(K[4][i], D::E4)),
                                 pm(K[5][i], D::E5)),
                              pm(K[6][i], D::E6));
        err[i] = pm(e, h);
      }
      const double en = rms4_div(err, sc);
      if (en < 1.0) {
        double factor = en == 0.0 ? 10.0 : fmin(10.0, pm(0.9, pow(en, -0.2)));
        if (rejected) factor = fmin(1.0, factor);
        h_abs = pm(h_abs, factor);
        break;
      }
      h_abs = pm(h_abs, fmax(0.2, pm(0.9, pow(en, -0.2))));
      rejected = true;
    }
    t = t_new;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[i] = ynew[i];
      f[i] = K[6][i];
    }
    if (ps(t, t1) >= 0) return true;
  }
}

}  // namespace mpcqp
