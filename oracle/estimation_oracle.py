"""CPU restatements of the estimator and the nonlinear plant around the closed loop
(TEST INFRASTRUCTURE ONLY: imported by tests/, tests/golden/gen_fixtures_loops.py and
__graft_entry__.smoke(); never by the product).

* `MerweScaledSigmaPoints`, `UnscentedKalmanFilter`, `unscented_transform` -- filterpy 1.4.5
  (filterpy/kalman/sigma_points.py, UKF.py, unscented_transform.py), restated with numpy in the
  same operation order.  The reference imports filterpy (src/trajectorySimulate.py:13,
  src/trajectorySimulateC.py:13) but neither vendors it nor is it installed here, so parity with
  filterpy itself is UNPINNED; the reference's own loops are pinned around this restatement
  (tests/golden/cl_noise_n20.npz).
* `state_eqn_n`, `plant_substep` -- reference src/trajectorySimulateC.py:64-79 and :373-380,
  integrated by the real scipy.integrate.solve_ivp (installed here and on the GPU box): pinned.
"""
from __future__ import annotations

import numpy as np
import scipy.integrate
import scipy.linalg


class MerweScaledSigmaPoints:
    """filterpy.kalman.MerweScaledSigmaPoints (sqrt_method = scipy.linalg.cholesky, upper)."""

    def __init__(self, n, alpha, beta, kappa=0.0):
        self.n, self.alpha, self.beta, self.kappa = n, alpha, beta, kappa
        self._compute_weights()

    def num_sigmas(self):
        return 2 * self.n + 1

    def sigma_points(self, x, P):
        n = self.n
        x = np.asarray(x, dtype=float)
        P = np.atleast_2d(P)
        lambda_ = self.alpha ** 2 * (n + self.kappa) - n
        U = scipy.linalg.cholesky((lambda_ + n) * P)
        sigmas = np.zeros((2 * n + 1, n))
        sigmas[0] = x
        for k in range(n):
            sigmas[k + 1] = np.subtract(x, -U[k])
            sigmas[n + k + 1] = np.subtract(x, U[k])
        return sigmas

    def _compute_weights(self):
        n = self.n
        lambda_ = self.alpha ** 2 * (n + self.kappa) - n
        c = .5 / (n + lambda_)
        self.Wc = np.full(2 * n + 1, c)
        self.Wm = np.full(2 * n + 1, c)
        self.Wc[0] = lambda_ / (n + lambda_) + (1 - self.alpha ** 2 + self.beta)
        self.Wm[0] = lambda_ / (n + lambda_)


def unscented_transform(sigmas, Wm, Wc, noise_cov=None):
    """filterpy.kalman.unscented_transform, default mean / residual (np.subtract) path."""
    x = np.dot(Wm, sigmas)
    y = sigmas - x[np.newaxis, :]
    P = np.dot(y.T, np.dot(np.diag(Wc), y))
    if noise_cov is not None:
        P += noise_cov
    return x, P


class UnscentedKalmanFilter:
    """filterpy.kalman.UnscentedKalmanFilter: the predict / update pair the reference calls.

    The reference's fx takes (x, u) and it calls kf.predict(ctrls[:, i]): the control lands in
    filterpy's `dt` argument and is passed on as fx(sigma, dt) (src/trajectorySimulate.py:121,334).
    """

    def __init__(self, dim_x, dim_z, dt, hx, fx, points):
        self.x = np.zeros(dim_x)
        self.P = np.eye(dim_x)
        self.Q = np.eye(dim_x)
        self._dim_x, self._dim_z, self._dt = dim_x, dim_z, dt
        self.points_fn = points
        self._num_sigmas = points.num_sigmas()
        self.hx, self.fx = hx, fx
        self.Wm, self.Wc = points.Wm, points.Wc
        self.R = np.eye(dim_z)
        self.sigmas_f = np.zeros((self._num_sigmas, dim_x))
        self.sigmas_h = np.zeros((self._num_sigmas, dim_z))

    def predict(self, dt=None, fx=None, **fx_args):
        if dt is None:
            dt = self._dt
        fx = fx or self.fx
        sigmas = self.points_fn.sigma_points(self.x, self.P)
        for i, s in enumerate(sigmas):
            self.sigmas_f[i] = fx(s, dt, **fx_args)
        self.x, self.P = unscented_transform(self.sigmas_f, self.Wm, self.Wc, self.Q)
        self.sigmas_f = self.points_fn.sigma_points(self.x, self.P)
        self.x_prior, self.P_prior = np.copy(self.x), np.copy(self.P)

    def update(self, z, R=None, hx=None, **hx_args):
        hx = hx or self.hx
        if R is None:
            R = self.R
        elif np.isscalar(R):
            R = np.eye(self._dim_z) * R
        self.sigmas_h = np.atleast_2d([hx(s, **hx_args) for s in self.sigmas_f])
        zp, self.S = unscented_transform(self.sigmas_h, self.Wm, self.Wc, R)
        self.SI = np.linalg.inv(self.S)
        Pxz = np.zeros((self.sigmas_f.shape[1], self.sigmas_h.shape[1]))
        for i in range(self.sigmas_f.shape[0]):
            dx = np.subtract(self.sigmas_f[i], self.x)
            dz = np.subtract(self.sigmas_h[i], zp)
            Pxz += self.Wc[i] * np.outer(dx, dz)
        self.K = np.dot(Pxz, self.SI)
        self.y = np.subtract(z, zp)
        self.x = self.x + np.dot(self.K, self.y)
        self.P = self.P - np.dot(self.K, np.dot(self.S, self.K.T))


def reference_ukf(Ao, Bou, Q, R, x0, P0, alpha=0.1, beta=2., kappa=-1):
    """the filter exactly as the reference sets it up (src/trajectorySimulate.py:113-130,271-278)"""
    import math

    def fx(x, u):
        return Ao @ x + Bou @ u

    def hx(x):
        ymeas = np.empty(2)
        ymeas[0] = np.linalg.norm(x[:2])
        ymeas[1] = math.atan2(x[1], x[0])
        return ymeas

    kf = UnscentedKalmanFilter(dim_x=6, dim_z=2, dt=None, fx=fx, hx=hx,
                               points=MerweScaledSigmaPoints(6, alpha=alpha, beta=beta, kappa=kappa))
    kf.x = np.array(x0, dtype=float)
    kf.P = np.array(P0, dtype=float)
    kf.R = np.array(R, dtype=float)
    kf.Q = np.array(Q, dtype=float)
    return kf


def state_eqn_n(n):
    """reference src/trajectorySimulateC.py:64-79 (closure over the mean motion n)"""

    def stateEqnN(t, x, u):
        h = 500e+03
        re = 6378.1e+03
        R_T = h + re
        mu = (n ** 2) * (R_T ** 3)
        dxdt = [None] * 4
        dxdt[0] = x[2]
        dxdt[1] = x[3]
        dxdt[2] = 2 * n * x[3] + (n ** 2) * x[0] - (mu * (R_T + x[0])) / (((R_T + x[0]) ** 2 + x[1] ** 2) ** (3 / 2)) + mu / (R_T ** 2) + u[0]
        dxdt[3] = -2 * n * x[2] + (n ** 2) * x[1] - (mu * x[1]) / (((R_T + x[0]) ** 2 + x[1] ** 2) ** (3 / 2)) + u[1]
        return dxdt

    return stateEqnN


def plant_substep(n, x, u, t, dt):
    """x(t + dt) of the nonlinear plant as the reference integrates it (solve_ivp defaults)"""
    soln = scipy.integrate.solve_ivp(state_eqn_n(n), (t, t + dt), np.asarray(x, dtype=float),
                                     args=(np.asarray(u, dtype=float),))
    return soln.y[:, -1], soln.status
