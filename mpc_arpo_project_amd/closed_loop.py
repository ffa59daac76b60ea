"""Batched, device-resident closed loops of the reference's simulators.

`BatchClosedLoop` advances B independent chasers through the discrete-time loop
(reference src/trajectorySimulate.py:285-356) entirely on the GPU:

    solve (HIP engine, warm-started)  ->  controller select + clip + CW plant  (mpcqp_cl_step)
                                      ->  UKF predict + update (noise != None)  (mpcqp_ukf_step)
                                      ->  configureDynamicConstraints          (mpcqp_cl_configure)
                                      ->  noise redraw every noise_length steps (mpcqp_cl_noise)

`BatchClosedLoopC` does the same for the continuous-time nonlinear loop
(src/trajectorySimulateC.py:325-409): one `period()` is a solve at a sample instant followed by
the RK45 plant sub-steps up to the next sample (mpcqp_clc_period).

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


def _noise_params(noise):
    """(sig_x, sig_y, noise_length) from a Noise object or a tuple; None -> None"""
    if noise is None:
        return None
    if hasattr(noise, "noise_std"):
        return float(noise.noise_std[0]), float(noise.noise_std[1]), noise.noise_length
    sx, sy, rep = noise
    return float(sx), float(sy), rep


class BatchClosedLoop:
    """B chasers of one scenario family stepping through the closed loop on one GPU.

    noise: None (the reference's noise=None path: perfect state feedback) or a Noise /
    (sig_x, sig_y, noise_length): plant noise plus the UKF estimator, as the reference does when
    noise is not None.  noise_source: None draws noiseVec on the device from a counter-based
    stream keyed by (noise_seed, global chaser id = id_offset + b, draw index); a callable
    draw(k) -> (B, 4) array supplies draw k from the host instead (e.g. numpy's seeded global
    generator, for parity with the reference's own runs).
    """

    def __init__(self, prob: MPCProblem, x0, device="cuda", noise=None, noise_seed=123,
                 id_offset=0, noise_source=None, longest_first=False, **settings):
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
        self.aborted = torch.zeros(self.B, dtype=torch.int32, device=self.device)
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
        # terminated chasers are not solved again (the reference leaves its loop at termination)
        self.qp.set_skip(self.done)
        # solve order (longest_first=True): every step after the first hands the chasers to the
        # persistent launch longest-first by their last solve's ADMM iterations (a warm closed
        # loop's best predictor of the next), so the max_iter runs start first and the launch ends
        # on short solves (results unchanged, mpcqp_set_order).  Off by default: on the bench it
        # measured 896k vs 895k solves/s with two shards and 798k vs 807k with one
        # (profiles/r03/ab_order.txt) -- the launch's tail is not where the time goes
        self._order = None
        if longest_first:
            self._order = torch.arange(self.B, dtype=torch.int32, device=self.device)
            self.qp.set_order(self._order)
        self.u0 = prob.u0_slice.start
        self.steps = 0
        check(_lib.lib().mpcqp_cl_set_ids(self._cl, int(id_offset)), "mpcqp_cl_set_ids")
        self._init_noise(noise, noise_seed, noise_source, xest, noise_dt=None)

    def _init_noise(self, noise, seed, source, xest0, noise_dt):
        self.noise = _noise_params(noise)
        self.noise_seed, self._noise_source = int(seed), source
        self.ukf = None
        self.w = self.z = self.u_applied = None
        if self.noise is None:
            return
        from .estimation import BatchUKF, observer_model

        f = dict(dtype=torch.float64, device=self.device)
        self.w = torch.zeros(self.B, 4, **f)
        self.z = torch.zeros(self.B, 2, **f)
        self.u_applied = torch.zeros(self.B, 2, **f)
        Ao, Bou, Qw, R, P0 = observer_model(self.prob, self.noise[:2], noise_dt)
        self.ukf = BatchUKF(Ao, Bou, Qw, R, xest0, P0, device=self.device, stream=self.qp.stream)
        self._draw(0)

    def _draw(self, k):
        """noiseVec draw k into self.w (async on the engine stream)"""
        if self._noise_source is not None:
            w = np.asarray(self._noise_source(k), dtype=float).reshape(self.B, 4)
            with torch.cuda.stream(self.qp.stream):
                self.w.copy_(torch.as_tensor(w), non_blocking=False)
            return
        sx, sy = self._noise_scale()
        check(_lib.lib().mpcqp_cl_noise(self._cl, self.noise_seed, int(k), sx, sy,
                                        self.w.data_ptr()), "mpcqp_cl_noise")

    def _noise_scale(self):
        return self.noise[0], self.noise[1]

    def _estimate(self):
        """UKF step on the measurement the plant kernel produced, estimate -> xest.  A chaser whose
        UKF covariance stops being positive definite is frozen as aborted: filterpy raises
        numpy.linalg.LinAlgError there and the reference's run ends with that exception."""
        self.ukf.step(self.u_applied, self.z, active=self.ctrl_seq)
        with torch.cuda.stream(self.qp.stream):
            self.xest.copy_(self.ukf.x)
            bad = ((self.ukf.status != 0) & (self.done == 0)).to(torch.int32)
            self.aborted.bitwise_or_(bad)
            self.done.bitwise_or_(bad)
            if getattr(self, "_tracking", False):
                self.iterm.copy_(torch.where(bad > 0, self.steps + 1, self.iterm))

    def step(self):
        """Solve the current QPs, apply the controller and plant, rebuild the QP data (async)."""
        return self.step_after_solve(self.qp.solve_async())

    def enable_tracking(self, nsim, dist_tol=0.2, ang_tol=45.0):
        """Keep the per-chaser run summary on the device from now on (call before the first step):
        the reference's run reduction -- i_term, isSuccess (src/trajectorySimulate.py:288-293,
        369-376), the final error |x(i_term - 1) - xr| of test/disturbRejComp.py:88 -- plus the
        first MPC input, the last solve status, total ADMM iterations and fallback-step count.
        `summary()` packs them."""
        if self.steps:
            raise MPCQPError("enable_tracking must precede the first step")
        i32 = dict(dtype=torch.int32, device=self.device)
        self.iterm = torch.where(self.done > 0, 0, int(nsim)).to(torch.int32).contiguous()
        self.success = torch.zeros(self.B, **i32)
        self.n_fallback = torch.zeros(self.B, **i32)
        self.final_err = torch.zeros(self.B, dtype=torch.float64, device=self.device)
        self.iters_total = torch.zeros(self.B, dtype=torch.int64, device=self.device)
        self.last_status = torch.zeros(self.B, **i32)
        self.u0_first = torch.full((self.B, 2), float("nan"), dtype=torch.float64,
                                   device=self.device)
        check(_lib.lib().mpcqp_cl_set_tracking(self._cl, self.iterm.data_ptr(),
                                               self.success.data_ptr(), self.final_err.data_ptr(),
                                               self.n_fallback.data_ptr(), float(dist_tol),
                                               float(ang_tol)), "mpcqp_cl_set_tracking")
        self._tracking = True

    SUMMARY_FIELDS = ("u0_x", "u0_y", "last_status", "admm_iters", "i_term", "success",
                      "final_err", "n_fallback", "aborted")

    def summary(self):
        """(B, 9) float64 device tensor, columns SUMMARY_FIELDS (ordered after this loop's stream)"""
        if not getattr(self, "_tracking", False):
            raise MPCQPError("enable_tracking() first")
        torch.cuda.current_stream(self.device).wait_stream(self.qp.stream)
        return torch.cat([self.u0_first, self.last_status[:, None].double(),
                          self.iters_total[:, None].double(), self.iterm[:, None].double(),
                          self.success[:, None].double(), self.final_err[:, None],
                          self.n_fallback[:, None].double(), self.aborted[:, None].double()],
                         dim=1)

    def _track_solve(self, r):
        with torch.cuda.stream(self.qp.stream):
            active = self.done == 0
            self.iters_total += torch.where(active, r.iter, 0).to(torch.int64)
            self.last_status.copy_(torch.where(active, r.status, self.last_status))
            if self.steps == 0:
                u = r.x[:, self.u0:self.u0 + 2]
                self.u0_first.copy_(torch.where(active[:, None], u, self.u0_first))

    def _reorder(self, r):
        """next solve's order: longest-first by this solve's ADMM iterations (engine stream)"""
        if self._order is not None:
            with torch.cuda.stream(self.qp.stream):
                self._order.copy_(torch.argsort(r.iter, descending=True))

    def step_after_solve(self, r):
        """Controller select + plant + QP-data rebuild for a solve already enqueued (async)."""
        L = _lib.lib()
        if getattr(self, "_tracking", False):
            self._track_solve(r)
        self._reorder(r)
        opt = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        rc = L.mpcqp_cl_step(self._cl, r.status.data_ptr(), r.x.data_ptr(), self.qp.n, self.u0,
                             self.x_true.data_ptr(), self.ctrl_prev.data_ptr(),
                             self.xintf.data_ptr(), self.xest.data_ptr(), self.done.data_ptr(),
                             self.ctrl_seq.data_ptr(), self.ctrl.data_ptr(), opt(self.w),
                             opt(self.z), opt(self.u_applied))
        if rc:
            raise MPCQPError(f"mpcqp_cl_step failed ({rc})")
        if self.ukf is not None:
            self._estimate()
        ax, l, u = self._bufs
        rc = L.mpcqp_cl_configure(self._cl, self.xest.data_ptr(), ax, l, u)
        if rc:
            raise MPCQPError(f"mpcqp_cl_configure failed ({rc})")
        self.steps += 1
        if self.noise is not None and self.steps % self.noise[2] == 0:
            self._draw(self.steps // int(self.noise[2]))
        return r

    def close(self):
        if getattr(self, "_cl", None):
            self.qp.stream.synchronize()
            _lib.lib().mpcqp_cl_destroy(self._cl)
            self._cl = None
        if getattr(self, "ukf", None) is not None:
            self.ukf.close()
        self.qp.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_SHARD_STREAMS = {}


def shard_streams(device, S):
    """S HIP streams for S concurrent shards, the same ones for every sharded loop of the process.
    Fresh pool streams per loop let two shards of a later loop land on one hardware queue (the
    process has GPU_MAX_HW_QUEUES = 4), and then their launches run one after the other: the
    default bench's first N = 40 leg took 232 ms per step for two 116 ms launches while the
    headline's two shards overlapped (Measured).  Reusing the first loop's streams keeps
    every later loop on the queue assignment the first one had."""
    import torch

    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    have = _SHARD_STREAMS.setdefault(key, [])
    while len(have) < S:
        have.append(torch.cuda.Stream(device=dev))
    return have[:S]


class ShardedClosedLoop:
    """A BatchClosedLoop split into S shards of consecutive chasers, each on its own HIP stream.

    The solve kernel of one launch ends with a tail (the few instances that run to max_iter keep a
    handful of CUs busy); with S = 2 the other shard's launch fills the idle CUs, so a K-step sweep
    runs ~10 % faster than one batch on one stream (Measured).  Results are identical to
    the unsharded loop: chasers are independent and keep their global ids (noise streams).
    """

    def __init__(self, prob: MPCProblem, x0, shards=2, device="cuda", id_offset=0,
                 noise_source=None, **kw):
        x0 = np.asarray(x0, dtype=float)
        B = x0.shape[0]
        S = max(1, min(int(shards), B))
        self.cut = [B * j // S for j in range(S + 1)]
        dev = torch.device(device)
        self.parts = []
        # a host noise source draws for the WHOLE batch (e.g. numpy's seeded global generator):
        # draw k once, cache it, hand each shard its rows, so the host RNG advances exactly as in
        # the unsharded loop
        self._draw_k, self._draw_w = None, None

        def shard_source(j):
            if noise_source is None:
                return None

            def draw(k, a=self.cut[j], b=self.cut[j + 1]):
                if self._draw_k != k:
                    self._draw_w = np.asarray(noise_source(k), dtype=float).reshape(B, 4)
                    self._draw_k = k
                return self._draw_w[a:b]
            return draw

        sts = shard_streams(dev, S) if S > 1 else [None]
        for j in range(S):
            self.parts.append(BatchClosedLoop(prob, x0[self.cut[j]:self.cut[j + 1]], device=dev,
                                              id_offset=id_offset + self.cut[j], stream=sts[j],
                                              noise_source=shard_source(j), **kw))
        torch.cuda.synchronize(dev)

    def step(self):
        """One closed-loop step of every shard, enqueued shard after shard (async)."""
        return [c.step() for c in self.parts]

    def _cat(self, name):
        # each shard writes its buffers on its own stream: order the caller's stream after them
        cur = torch.cuda.current_stream(self.parts[0].device)
        for c in self.parts:
            cur.wait_stream(c.qp.stream)
        return torch.cat([getattr(c, name) for c in self.parts])

    def enable_tracking(self, nsim, dist_tol=0.2, ang_tol=45.0):
        for c in self.parts:
            c.enable_tracking(nsim, dist_tol, ang_tol)

    SUMMARY_FIELDS = BatchClosedLoop.SUMMARY_FIELDS

    def summary(self):
        return torch.cat([c.summary() for c in self.parts])

    @property
    def x_true(self):
        return self._cat("x_true")

    @property
    def done(self):
        return self._cat("done")

    @property
    def ctrl_seq(self):
        return self._cat("ctrl_seq")

    def synchronize(self):
        for c in self.parts:
            c.qp.stream.synchronize()

    def close(self):
        for c in self.parts:
            c.close()


def sample_schedule(T, T_cont, T_final, i0=500):
    """The sample periods of trajectorySimulateC's loop (src/trajectorySimulateC.py:323-409):
    [(i_start, nsub, time at i_start)], the loop index starting at the literal 500, a sample
    where `disc_j < nsimD and xTimeC[i] == xTimeD[disc_j]`, `time` accumulated by repeated
    addition of T_cont from T, exactly as the reference does."""
    nsimD = int(T_final / T)
    nsimC = int(T_final / T_cont)
    xTimeD = np.arange(0, T_final, T)
    xTimeC = np.arange(0, T_final, T_cont)
    out = []
    disc_j, time = 1, T
    for i in range(i0, nsimC - 1):
        if disc_j < nsimD and xTimeC[i] == xTimeD[disc_j]:
            out.append([i, 0, time])
            disc_j += 1
        elif not out:
            raise MPCQPError("the first loop iteration of trajectorySimulateC must be a sample")
        out[-1][1] += 1
        time = time + T_cont
    return [tuple(p) for p in out]


class BatchClosedLoopC(BatchClosedLoop):
    """B chasers through the continuous-time nonlinear loop of trajectorySimulateC on one GPU.

    `period()` = the solve at a sample instant + the RK45 plant sub-steps up to the next sample
    (+ UKF and QP rebuild when noise is given).  `iterm` holds the loop index at which a chaser's
    termination test fired (nsimC if it never did).  The continuous-time noise of the reference
    (python-control white_noise with covariance Qcont / 0.001, held for noise_length samples) is
    drawn from the device stream with that covariance; python-control is absent here, so its exact
    draws are not reproduced.
    """

    def __init__(self, prob: MPCProblem, x0, T_cont, T_final, mean_motion, isDeltaV=False,
                 device="cuda", noise=None, noise_seed=123, id_offset=0, noise_source=None,
                 **settings):
        super().__init__(prob, x0, device=device, noise=None, **settings)
        from .estimation import plant_model

        self.T_cont, self.T_final = float(T_cont), float(T_final)
        self.schedule = sample_schedule(prob.T, self.T_cont, self.T_final)
        self.nsimC = int(self.T_final / self.T_cont)
        self._plant = plant_model(mean_motion)
        check(_lib.lib().mpcqp_cl_set_plant(self._cl, C.byref(self._plant), int(bool(isDeltaV))),
              "mpcqp_cl_set_plant")
        check(_lib.lib().mpcqp_cl_set_ids(self._cl, int(id_offset)), "mpcqp_cl_set_ids")
        self.iterm = torch.full((self.B,), self.nsimC, dtype=torch.int32, device=self.device)
        xest = self.xest.cpu().numpy()
        if prob.inTrack:
            xest[:, [0, 1]] = xest[:, [1, 0]]
        hold = int(prob.T / self.T_cont)
        self._init_noise(noise, noise_seed, noise_source, xest, noise_dt=prob.T * hold)
        self.period_index = 0

    def enable_tracking(self, nsim, dist_tol=0.2, ang_tol=45.0):
        """Not available for the continuous loop: mpcqp_clc_period keeps i_term (self.iterm) but
        not the success / final-error / fallback run summary of the discrete loop's tracking."""
        raise NotImplementedError("run summaries are tracked by the discrete loop only; "
                                  "BatchClosedLoopC exposes iterm, done and ctrl_seq")

    def _noise_scale(self):
        s = 1.0 / np.sqrt(0.001)
        return self.noise[0] * s, self.noise[0] * s  # Qcont = diag(sig_x^2, sig_x^2) (quirk)

    @property
    def periods(self):
        return len(self.schedule)

    def period(self, traj=None, on_solved=None):
        """One sample period for every chaser (async); traj: optional (B, nsub, 4) tensor;
        on_solved(stream): called right after the solve is enqueued (e.g. an event record, to
        split the period's time between the solve and the plant / UKF / configure work)"""
        if self.period_index >= len(self.schedule):
            raise MPCQPError("the simulation horizon is exhausted")
        i0, nsub, t0 = self.schedule[self.period_index]
        r = self.qp.solve_async()
        if on_solved is not None:
            on_solved(self.qp.stream)
        self._reorder(r)
        L = _lib.lib()
        opt = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        if traj is not None and (tuple(traj.shape) != (self.B, nsub, 4) or
                                 traj.dtype != torch.float64 or not traj.is_contiguous()):
            raise ValueError("traj must be a contiguous (B, nsub, 4) float64 tensor")
        check(L.mpcqp_clc_period(self._cl, r.status.data_ptr(), r.x.data_ptr(), self.qp.n,
                                 self.u0, self.x_true.data_ptr(), self.ctrl_prev.data_ptr(),
                                 self.xintf.data_ptr(), self.xest.data_ptr(),
                                 self.done.data_ptr(), self.iterm.data_ptr(),
                                 self.ctrl_seq.data_ptr(), self.ctrl.data_ptr(), opt(self.w),
                                 opt(self.z), opt(self.u_applied), t0, self.T_cont, i0, nsub,
                                 opt(traj)), "mpcqp_clc_period")
        if self.ukf is not None:
            self._estimate()
        ax, l, u = self._bufs
        check(L.mpcqp_cl_configure(self._cl, self.xest.data_ptr(), ax, l, u),
              "mpcqp_cl_configure")
        self.period_index += 1
        if self.noise is not None and self.period_index % int(self.noise[2]) == 0:
            self._draw(self.period_index // int(self.noise[2]))
        return r


class ShardedClosedLoopC:
    """A BatchClosedLoopC split into S shards of consecutive chasers, each on its own HIP stream
    (ShardedClosedLoop for the continuous-time loop): while one shard's solve launch runs out its
    tail (config 4's solves run up to max_iter: p90 2,300 ADMM iterations against a mean of ~570),
    the other shard's solve, plant sub-steps and UKF fill the idle CUs.  Results are identical to
    the unsharded loop: chasers are independent and keep their global ids (device noise streams,
    mpcqp_cl_set_ids)."""

    def __init__(self, prob: MPCProblem, x0, T_cont, T_final, mean_motion, shards=2, device="cuda",
                 id_offset=0, noise_source=None, **kw):
        x0 = np.asarray(x0, dtype=float)
        B = x0.shape[0]
        S = max(1, min(int(shards), B))
        self.cut = [B * j // S for j in range(S + 1)]
        dev = torch.device(device)
        self._draw_k, self._draw_w = None, None

        def shard_source(j):
            if noise_source is None:
                return None

            def draw(k, a=self.cut[j], b=self.cut[j + 1]):
                if self._draw_k != k:
                    self._draw_w = np.asarray(noise_source(k), dtype=float).reshape(B, 4)
                    self._draw_k = k
                return self._draw_w[a:b]
            return draw

        sts = shard_streams(dev, S) if S > 1 else [None]
        self.parts = [BatchClosedLoopC(prob, x0[self.cut[j]:self.cut[j + 1]], T_cont, T_final,
                                       mean_motion, device=dev, id_offset=id_offset + self.cut[j],
                                       stream=sts[j], noise_source=shard_source(j), **kw)
                      for j in range(S)]
        self.B = B
        self.schedule = self.parts[0].schedule
        self.nsimC = self.parts[0].nsimC
        self.qp = self.parts[0].qp  # schedule_info / dims (the same plan in every shard)
        torch.cuda.synchronize(dev)

    @property
    def periods(self):
        return self.parts[0].periods

    @property
    def period_index(self):
        return self.parts[0].period_index

    def period(self, on_solved=None):
        """One sample period of every shard, enqueued shard after shard (async); the solve results
        of the shards (on_solved(stream) is called after each shard's solve is enqueued)"""
        return [c.period(on_solved=on_solved) for c in self.parts]

    def _cat(self, name):
        cur = torch.cuda.current_stream(self.parts[0].device)
        for c in self.parts:
            cur.wait_stream(c.qp.stream)
        return torch.cat([getattr(c, name) for c in self.parts])

    @property
    def x_true(self):
        return self._cat("x_true")

    @property
    def done(self):
        return self._cat("done")

    @property
    def iterm(self):
        return self._cat("iterm")

    @property
    def ctrl_seq(self):
        return self._cat("ctrl_seq")

    def synchronize(self):
        for c in self.parts:
            c.qp.stream.synchronize()

    def close(self):
        for c in self.parts:
            c.close()
