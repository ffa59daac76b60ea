"""Batched, device-resident closed loop of the discrete-time linear simulator.

One `BatchClosedLoop` advances B independent chasers through the reference's control loop
(reference src/trajectorySimulate.py:285-356, noise=None path) entirely on the GPU:

    solve (HIP engine, warm-started)  ->  controller select + clip + CW plant  (mpcqp_cl_step)
                                      ->  configureDynamicConstraints          (mpcqp_cl_configure)

The per-step QP data never leaves HBM: the configure kernel rewrites the varying A values and
bounds in the engine's own buffers.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import MPCQPError, check
from .engine import BatchQP, data_buffers
from .qp_model import MPCProblem, configure_batch


def scenario_struct(prob: MPCProblem):
    """Host description of the scenario for the closed-loop kernels (keeps the index arrays alive
    through the returned tuple)."""
    if (prob.nx, prob.nu, prob.ny, prob.ndi) != (4, 2, 5, 2):
        raise MPCQPError("the closed-loop kernels implement the planar CW model (4, 2, 5, 2)")
    if prob.Kpf is None:
        raise MPCQPError("build_problem(..., fail_params) is required for the fallback gains")
    sc = _lib.ClScenario()
    sc.Nx, sc.Nc, sc.Nb, sc.m, sc.nnzA = prob.Nx, prob.Nc, prob.Nb, prob.m, prob.nnzA
    sc.Ad[:] = [float(v) for v in np.asarray(prob.Ad).ravel()]
    sc.Bd[:] = [float(v) for v in np.asarray(prob.Bd).ravel()]
    sc.rp, sc.rtol = prob.rp, prob.rtol
    sc.xr[:] = [float(v) for v in prob.xr]
    sc.inTrack, sc.isReject, sc.has_debris = int(prob.inTrack), int(prob.isReject), int(prob.has_debris)
    if prob.has_debris:
        sc.center[:] = [float(prob.center[0]), float(prob.center[1])]
        sc.verts[:] = [float(v) for v in np.asarray(prob.verts).ravel()]
    else:
        sc.center[:] = [-np.inf, -np.inf]
    sc.side, sc.detect = float(prob.side), float(prob.detect)
    sc.umin[:] = [float(v) for v in prob.umin]
    sc.umax[:] = [float(v) for v in prob.umax]
    sc.Kpf[:] = [float(v) for v in np.asarray(prob.Kpf).ravel()]
    sc.Kif[:] = [float(v) for v in np.asarray(prob.Kif).ravel()]
    sc.Ktot[:] = [float(v) for v in np.asarray(prob.K_total).ravel()]
    sc.Ki[:] = [float(v) for v in np.asarray(prob.K_i).ravel()]
    sc.Crefx[:] = [float(v) for v in np.asarray(prob.Crefx).ravel()]
    sc.Crefy[:] = [float(v) for v in np.asarray(prob.Crefy).ravel()]
    keep = [np.ascontiguousarray(prob.pos_c1, dtype=np.int32),
            np.ascontiguousarray(prob.pos_c2, dtype=np.int32)]
    sc.pos_c1 = keep[0].ctypes.data_as(C.POINTER(C.c_int32))
    sc.pos_c2 = keep[1].ctypes.data_as(C.POINTER(C.c_int32))
    if len(prob.pos_slope):
        keep.append(np.ascontiguousarray(prob.pos_slope, dtype=np.int32))
        sc.pos_slope = keep[2].ctypes.data_as(C.POINTER(C.c_int32))
    else:
        sc.pos_slope = C.POINTER(C.c_int32)()
    return sc, keep


class BatchClosedLoop:
    """B chasers of one scenario family stepping through the closed loop on one GPU."""

    def __init__(self, prob: MPCProblem, x0, device="cuda", **settings):
        x0 = np.asarray(x0, dtype=float)
        if x0.ndim != 2 or x0.shape[1] != 4:
            raise ValueError("x0 must have shape (B, 4)")
        self.prob = prob
        self.B = x0.shape[0]
        settings.setdefault("warm_start", True)
        self.qp = BatchQP(prob.P, prob.A, batch=self.B, device=device, **settings)
        self.device = self.qp.device
        xest = np.hstack([x0, np.zeros((self.B, 2))])  # xest0 = [x0, 0, 0] (src/...:249)
        Ax, l, u = configure_batch(prob, xest)
        self.qp.set_data(q=prob.q, Ax=Ax, l=l, u=u)
        f = dict(dtype=torch.float64, device=self.device)
        self.x_true = torch.as_tensor(x0, **f).contiguous()
        self.xest = torch.as_tensor(xest, **f).contiguous()
        if prob.inTrack:  # quirk Q4 applied by the initial configureDynamicConstraints call
            self.xest[:, [0, 1]] = self.xest[:, [1, 0]]
        self.ctrl_prev = torch.zeros(self.B, 2, **f)
        self.ctrl = torch.zeros(self.B, 2, **f)
        self.xintf = torch.zeros(self.B, **f)
        self.done = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.ctrl_seq = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        rn = np.hypot(x0[:, 0], x0[:, 1])
        pos = x0[:, 1] if prob.inTrack else x0[:, 0]
        self.done[:] = torch.as_tensor(((rn < prob.rp) | (pos < prob.rp - prob.rtol)).astype(np.int32))
        self._sc, self._keep = scenario_struct(prob)
        h = C.c_void_p()
        rc = _lib.lib().mpcqp_cl_create(C.byref(self._sc), self.B,
                                        C.c_void_p(self.qp.stream.cuda_stream), C.byref(h))
        if rc:
            raise MPCQPError(f"mpcqp_cl_create failed ({rc})")
        self._cl = h
        self._bufs = data_buffers(self.qp)
        self.u0 = prob.u0_slice.start
        self.steps = 0

    def step(self):
        """Solve the current QPs, apply the controller and plant, rebuild the QP data (async)."""
        return self.step_after_solve(self.qp.solve_async())

    def step_after_solve(self, r):
        """Controller select + plant + QP-data rebuild for a solve already enqueued (async)."""
        L = _lib.lib()
        rc = L.mpcqp_cl_step(self._cl, r.status.data_ptr(), r.x.data_ptr(), self.qp.n, self.u0,
                             self.x_true.data_ptr(), self.ctrl_prev.data_ptr(),
                             self.xintf.data_ptr(), self.xest.data_ptr(), self.done.data_ptr(),
                             self.ctrl_seq.data_ptr(), self.ctrl.data_ptr())
        if rc:
            raise MPCQPError(f"mpcqp_cl_step failed ({rc})")
        ax, l, u = self._bufs
        rc = L.mpcqp_cl_configure(self._cl, self.xest.data_ptr(), ax, l, u)
        if rc:
            raise MPCQPError(f"mpcqp_cl_configure failed ({rc})")
        self.steps += 1
        return r

    def close(self):
        if getattr(self, "_cl", None):
            self.qp.stream.synchronize()
            _lib.lib().mpcqp_cl_destroy(self._cl)
            self._cl = None
        self.qp.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
