"""Device-side state estimator and nonlinear plant (C ABI: include/mpcqp_estimation.h).

* `BatchUKF` -- B independent unscented Kalman filters of the reference's observer
  (src/trajectorySimulate.py:113-130,271-282,329-337; src/trajectorySimulateC.py:140-157,310-320,
  384-392): fx(x, u) = Ao x + Bou u, hx(x) = [|x[0:2]|, atan2(x[1], x[0])], sigma points
  MerweScaledSigmaPoints(6, 0.1, 2, -1).  One `step(u, z)` is filterpy's kf.predict(u) followed
  by kf.update(z), computed by `ukf_step_kernel` (csrc/estimation.hip).
* `UnscentedKalmanFilter` -- the single-instance object the simulators use in place of
  filterpy's (same attribute names x, P, Q, R; predict(u) records the input, update(z) runs the
  fused device step).
* `BatchPlant` -- the nonlinear relative-motion plant of trajectorySimulateC integrated with the
  restated scipy RK45 (`plant_rk45_kernel`), sub-step by sub-step like the reference's solve_ivp
  calls (src/trajectorySimulateC.py:64-79,371-380).

Everything runs on the GPU through libmpcqp.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.linalg
import torch

from . import _lib
from ._lib import MPCQPError


def observer_model(prob, noise_std=(0.0, 0.0), noise_dt=None):
    """(Ao, Bou, Q, R, P0) exactly as the reference builds them.

    Ao = blkdiag(Ad, I2) with the disturbance coupling Ao[0,4] = Ao[1,5] = 1, Bou = [Bd; 0]
    (src/trajectorySimulate.py:113-117); Q = Bnoise diag(sig^2) Bnoise' with Bnoise = [0; dt I2]
    and the quirky Q[:4, :4] = 0.001 I4 (:270-273; dt = T for the discrete loop, T * int(T/T_cont)
    for the continuous one, trajectorySimulateC.py:310-313); R = 0; P0 = blkdiag(1e-20 I4, I2).
    """
    nx, ndi = prob.nx, prob.ndi
    Ao = scipy.linalg.block_diag(np.asarray(prob.Ad), np.eye(ndi))
    Ao[0, 4] = 1.
    Ao[1, 5] = 1.
    Bou = np.vstack([np.asarray(prob.Bd), np.zeros([2, 2])])
    dt = prob.T if noise_dt is None else noise_dt
    sigMat = np.diag([noise_std[0], noise_std[1], 0, 0])
    Bnoise = np.vstack([np.zeros([nx, ndi]), dt * np.eye(ndi)])
    Qw = np.diag([sigMat[0, 0] ** 2, sigMat[1, 1] ** 2])
    Qw = Bnoise @ Qw @ np.transpose(Bnoise)
    Qw[:4, :][:, :4] = 0.001 * np.eye(nx)
    R = np.zeros([2, 2])
    P0 = scipy.linalg.block_diag(1e-20 * np.eye(nx), np.eye(ndi))
    return Ao, Bou, Qw, R, P0


def _ukf_struct(Ao, Bou, Q, R, alpha, beta, kappa):
    m = _lib.UkfModel()
    m.Ao[:] = [float(v) for v in np.asarray(Ao, dtype=float).ravel()]
    m.Bou[:] = [float(v) for v in np.asarray(Bou, dtype=float).ravel()]
    m.Q[:] = [float(v) for v in np.asarray(Q, dtype=float).ravel()]
    m.R[:] = [float(v) for v in np.asarray(R, dtype=float).ravel()]
    m.alpha, m.beta, m.kappa = float(alpha), float(beta), float(kappa)
    return m


def _device(device):
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def _stream_of(device, stream):
    if stream is not None:
        return stream
    return torch.cuda.current_stream(device)


class BatchUKF:
    """B filters on one GPU; state `x` (B, 6) and `P` (B, 6, 6) are float64 device tensors."""

    def __init__(self, Ao, Bou, Q, R, x0, P0, alpha=0.1, beta=2., kappa=-1, device="cuda",
                 stream=None):
        if not torch.cuda.is_available():
            raise MPCQPError("the UKF kernel needs a ROCm GPU (torch.cuda.is_available() is False)")
        x0 = np.atleast_2d(np.asarray(x0, dtype=float))
        if x0.shape[1] != 6 or np.shape(Ao) != (6, 6) or np.shape(Bou) != (6, 2):
            raise ValueError("the UKF kernel implements the 6-state / 2-input / 2-output observer")
        self.B = x0.shape[0]
        self.device = _device(device)
        self.stream = _stream_of(self.device, stream)
        f = dict(dtype=torch.float64, device=self.device)
        self.x = torch.as_tensor(x0, **f).contiguous()
        P0 = np.asarray(P0, dtype=float)
        P0 = np.broadcast_to(P0, (self.B, 6, 6)) if P0.ndim == 2 else P0
        self.P = torch.as_tensor(np.ascontiguousarray(P0), **f).contiguous()
        self.status = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self._model = _ukf_struct(Ao, Bou, Q, R, alpha, beta, kappa)
        h = C.c_void_p()
        rc = _lib.lib().mpcqp_ukf_create(C.byref(self._model), self.B,
                                         C.c_void_p(self.stream.cuda_stream), C.byref(h))
        if rc:
            raise MPCQPError(f"mpcqp_ukf_create failed ({rc})")
        self._h = h

    def step(self, u, z, active=None):
        """kf.predict(u); kf.update(z) for every instance (async on the stream); `u`, `z` are
        (B, 2) float64 device tensors, `active` an optional (B,) int32 mask."""
        for t in (u, z):
            if t.dtype != torch.float64 or t.device != self.device or t.shape != (self.B, 2) or \
                    not t.is_contiguous():
                raise ValueError("u and z must be contiguous (B, 2) float64 tensors on the device")
        act = None
        if active is not None:
            if active.dtype != torch.int32 or active.shape != (self.B,):
                raise ValueError("active must be a (B,) int32 tensor")
            act = C.c_void_p(active.data_ptr())
        rc = _lib.lib().mpcqp_ukf_step(self._h, C.c_void_p(self.x.data_ptr()),
                                       C.c_void_p(self.P.data_ptr()), C.c_void_p(u.data_ptr()),
                                       C.c_void_p(z.data_ptr()), act,
                                       C.c_void_p(self.status.data_ptr()))
        if rc:
            raise MPCQPError(f"mpcqp_ukf_step failed ({rc})")

    def close(self):
        if getattr(self, "_h", None):
            self.stream.synchronize()
            _lib.lib().mpcqp_ukf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class UnscentedKalmanFilter:
    """Single filter with filterpy's attribute names, stepped on the GPU.

    The reference always calls kf.predict(u) immediately followed by kf.update(z)
    (src/trajectorySimulate.py:334-335): predict records u, update runs the fused step.  Raises
    numpy.linalg.LinAlgError where filterpy's Cholesky would.
    """

    def __init__(self, Ao, Bou, Q, R, x0, P0, alpha=0.1, beta=2., kappa=-1, device="cuda"):
        self._k = BatchUKF(Ao, Bou, Q, R, np.asarray(x0)[None], np.asarray(P0)[None], alpha,
                           beta, kappa, device=device)
        self._u = None
        f = dict(dtype=torch.float64, device=self._k.device)
        self._ud = torch.zeros(1, 2, **f)
        self._zd = torch.zeros(1, 2, **f)

    @property
    def x(self):
        return self._k.x[0].cpu().numpy()

    @property
    def P(self):
        return self._k.P[0].cpu().numpy()

    def predict(self, u):
        self._u = np.asarray(u, dtype=float).reshape(2)

    def update(self, z):
        if self._u is None:
            raise RuntimeError("predict(u) must precede update(z)")
        self._ud.copy_(torch.as_tensor(self._u[None], dtype=torch.float64))
        self._zd.copy_(torch.as_tensor(np.asarray(z, dtype=float).reshape(1, 2)))
        self._k.step(self._ud, self._zd)
        self._u = None
        if int(self._k.status[0]) != 0:
            raise np.linalg.LinAlgError("UKF: (lambda + n) P is not positive definite")


def plant_model(mean_motion, rtol=1e-3, atol=1e-6):
    """stateEqnN's constants evaluated with the reference's Python-float expressions
    (src/trajectorySimulateC.py:67-77) and solve_ivp's default tolerances."""
    n = float(mean_motion)
    h = 500e+03
    re = 6378.1e+03
    R_T = h + re
    mu = (n ** 2) * (R_T ** 3)
    m = _lib.PlantModel()
    m.two_n, m.m_two_n, m.n2 = 2 * n, -2 * n, n ** 2
    m.R_T, m.mu, m.g0 = R_T, mu, mu / (R_T ** 2)
    m.rtol, m.atol = float(rtol), float(atol)
    return m


class BatchPlant:
    """RK45 integration of the nonlinear plant for B chasers (device tensors, float64)."""

    def __init__(self, mean_motion, batch, device="cuda", stream=None, rtol=1e-3, atol=1e-6):
        if not torch.cuda.is_available():
            raise MPCQPError("the plant kernel needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.B = int(batch)
        self.device = _device(device)
        self.stream = _stream_of(self.device, stream)
        self.model = plant_model(mean_motion, rtol, atol)
        self.failed = torch.zeros(self.B, dtype=torch.int32, device=self.device)

    def integrate(self, x, u, t0, dt, nsub, w=None, traj=None):
        """x <- nsub sub-steps of solve_ivp(stateEqnN, (t, t + dt), x, args=(u,)) + w, in place"""
        for t, shp in ((x, (self.B, 4)), (u, (self.B, 2))):
            if t.dtype != torch.float64 or t.device != self.device or tuple(t.shape) != shp or \
                    not t.is_contiguous():
                raise ValueError(f"expected a contiguous {shp} float64 device tensor")
        if w is not None and (w.shape != (self.B, 4) or w.dtype != torch.float64):
            raise ValueError("w must be a (B, 4) float64 tensor")
        if traj is not None and (tuple(traj.shape) != (self.B, nsub, 4) or
                                 traj.dtype != torch.float64 or not traj.is_contiguous()):
            raise ValueError("traj must be a contiguous (B, nsub, 4) float64 tensor")
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        rc = _lib.lib().mpcqp_plant_rk45(C.byref(self.model), self.B,
                                         C.c_void_p(self.stream.cuda_stream), ptr(x), ptr(u),
                                         ptr(w), float(t0), float(dt), int(nsub), ptr(traj),
                                         ptr(self.failed))
        if rc:
            raise MPCQPError(f"mpcqp_plant_rk45 failed ({rc})")
