"""Engine-driven vs oracle-driven full-length closed-loop runs (test infrastructure: imports the
oracle).  Both runs use the same device closed-loop kernels -- controller select + clip + CW plant,
UKF, configureDynamicConstraints, noise stream keyed by global scenario id -- which other tests pin
bit-exactly against the reference's runs; they differ only in who solves the per-step QPs:

  * engine-driven: the HIP engine (BatchClosedLoop.step);
  * oracle-driven: one OracleOSQP object per chaser (oracle/, the C restatement of OSQP 0.6),
    warm-started by itself step after step exactly as the reference's `prob` object is
    (reference src/trajectorySimulate.py:242-348: setup once, then update(l, u), update(Ax, l, u)
    and solve every step), fed the QP data the device configure kernel wrote and handing its
    (x, status) back to the device controller.

The runs are chaotic in the solver's rounding (one status flip changes the controller, and every
later state), so the comparison is made against the oracle's own floor: the oracle-driven run repeated from
initial states moved by one ulp, and with every solve's right-hand side moved by one ulp
(floor_run).  The reference's run reduction is compared:
isSuccess, i_term and the final distance |x(i_term - 1) - xr| (src/trajectorySimulate.py:359-387,
test/disturbRejComp.py:88)."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

import oracle as orc
from mpc_arpo_project_amd.closed_loop import BatchClosedLoop
from mpc_arpo_project_amd.engine import SolveResult

IDX = {k: i for i, k in enumerate(BatchClosedLoop.SUMMARY_FIELDS)}


def engine_run(prob, X0, nsim, suc_cond, noise, eps, noise_seed=123, id_offset=0):
    cl = BatchClosedLoop(prob, X0, noise=noise, noise_seed=noise_seed, id_offset=id_offset,
                         eps_abs=eps, eps_rel=eps)
    cl.enable_tracking(nsim, *suc_cond)
    for k in range(nsim):
        cl.step()
        if (k + 1) % 16 == 0 and bool(cl.done.all()):
            break
    out = cl.summary().cpu().numpy()
    cl.close()
    return out


class EngineKKT:
    """The engine's compiled device program on the CPU (libmpcqp mpcqp_emu_*: its factorization
    and blocked triangular solves, bitwise, tests/test_gpu_hybrid.py) as the oracle's KKT solver:
    attach(solver) gives one OracleOSQP its own solver state on the shared program."""

    def __init__(self, P, A):
        import ctypes as C

        from mpc_arpo_project_amd import _lib
        from mpc_arpo_project_amd.engine import sorted_csc, triu_csc

        self.L = _lib.lib()
        Pt, As = triu_csc(P), sorted_csc(A)
        self._arr = [np.ascontiguousarray(a, dtype=np.int32) for a in (Pt.indptr, Pt.indices,
                                                                        As.indptr, As.indices)]
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        st = _lib.Structure(Pt.shape[0], As.shape[0], *(ip(a) for a in self._arr))
        self._base = C.c_void_p()
        _lib.check(self.L.mpcqp_emu_create(C.byref(st), C.byref(self._base)), "mpcqp_emu_create")
        self._fac = C.cast(self.L.mpcqp_emu_factor, C.c_void_p).value
        self._sol = C.cast(self.L.mpcqp_emu_solve, C.c_void_p).value
        self._states = []

    def attach(self, solver, fused=False):
        import ctypes as C

        from mpc_arpo_project_amd import _lib

        h = C.c_void_p()
        _lib.check(self.L.mpcqp_emu_clone(self._base, C.byref(h)), "mpcqp_emu_clone")
        self._states.append(h)
        solver.set_kkt_hook(self._fac, self._sol, h.value)
        if fused:
            solver.set_fused_updates(True)

    def close(self):
        for h in self._states + [self._base]:
            self.L.mpcqp_emu_destroy(h)
        self._states, self._base = [], None


def oracle_run(prob, X0, nsim, suc_cond, noise, eps, noise_seed=123, id_offset=0, threads=16,
               jitter=0, solve_order=0, hybrid=0):
    """jitter != 0: every solver moves each KKT right-hand side by one ulp before each solve
    (oracle set_jitter, seeded per chaser); solve_order != 0: every solver's KKT solves sum each
    entry's products apart (oracle set_solve_order) -- floors of a different summation order.
    hybrid 1: every solver's KKT factorization and solves are the engine's compiled program
    (EngineKKT), OSQP's updates otherwise; 2: the same with the engine's fused ADMM updates
    (oracle set_fused_updates) -- the engine's arithmetic, bit for bit, on the CPU"""
    cl = BatchClosedLoop(prob, X0, noise=noise, noise_seed=noise_seed, id_offset=id_offset,
                         eps_abs=eps, eps_rel=eps)
    cl.enable_tracking(nsim, *suc_cond)
    B, n, m = cl.B, cl.qp.n, cl.qp.m
    dev = cl.device
    solvers = None
    f64 = dict(dtype=torch.float64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    for k in range(nsim):
        Ax, l, u = (t.cpu().numpy() for t in cl.qp.copy_data())
        act = np.flatnonzero((cl.done == 0).cpu().numpy())
        if act.size == 0:
            break
        if solvers is None:  # setup with the step-0 data (src/trajectorySimulate.py:242-245)
            solvers = []
            for b in range(B):
                A = sp.csc_matrix((Ax[b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
                s = orc.OracleOSQP()
                s.setup(prob.P, prob.q, A, l[b], u[b], eps_abs=eps, eps_rel=eps,
                        warm_start=True, verbose=False)
                if jitter:
                    s.set_jitter(jitter * 1000003 + b + 1)
                if solve_order:
                    s.set_solve_order(solve_order)
                if hybrid:
                    if b == 0:
                        ekkt = EngineKKT(prob.P, prob.A)
                    ekkt.attach(s, fused=hybrid == 2)
                solvers.append(s)
            x, st, it = orc.batch_update_solve([solvers[b] for b in act], None, None, None, threads)
        else:
            x, st, it = orc.batch_update_solve([solvers[b] for b in act], Ax[act], l[act], u[act],
                                               threads)
        X = np.full((B, n), np.nan)
        S = np.zeros(B, dtype=np.int32)
        It = np.zeros(B, dtype=np.int32)
        X[act], S[act], It[act] = x, st, it
        z = torch.zeros(B, **f64)
        r = SolveResult(x=torch.as_tensor(X, **f64), y=torch.zeros(B, m, **f64),
                        status=torch.as_tensor(S, **i32), iter=torch.as_tensor(It, **i32),
                        rho_updates=torch.zeros(B, **i32), obj_val=z, pri_res=z, dua_res=z, rho=z)
        torch.cuda.synchronize()
        cl.step_after_solve(r)
    out = cl.summary().cpu().numpy()
    cl.close()
    if hybrid and solvers:  # the solvers are done with their KKT states
        ekkt.close()
    return out


def compare(a, b):
    """agreement of two [G, 9] run summaries on the reference's run reduction"""
    sa, sb = a[:, IDX["success"]], b[:, IDX["success"]]
    ia, ib = a[:, IDX["i_term"]], b[:, IDX["i_term"]]
    fa, fb = a[:, IDX["final_err"]], b[:, IDX["final_err"]]
    same_run = (sa == sb) & (ia == ib) & (np.abs(fa - fb) <= 1e-6 * (1 + np.abs(fb)))
    # sampling noise of the differences of the reported statistics: paired bootstrap over the
    # scenarios (the same resampled chasers on both sides), standard error of the difference
    rng = np.random.default_rng(12345)
    idx = rng.integers(0, a.shape[0], size=(1000, a.shape[0]))
    se = dict(final_err_median=float(np.std(np.median(fa[idx], 1) - np.median(fb[idx], 1))),
              i_term_mean=float(np.std(ia[idx].mean(1) - ib[idx].mean(1))),
              success_rate=float(np.std(sa[idx].mean(1) - sb[idx].mean(1))))
    return dict(scenarios=int(a.shape[0]), se=se,
                success_rate=(float(sa.mean()), float(sb.mean())),
                success_agree=float(np.mean(sa == sb)),
                i_term_agree=float(np.mean(ia == ib)),
                i_term_mean=(float(ia.mean()), float(ib.mean())),
                final_err_median=(float(np.median(fa)), float(np.median(fb))),
                final_err_mean=(float(np.mean(fa)), float(np.mean(fb))),
                same_run=float(np.mean(same_run)))


FLOOR_DRAWS = 6


def floor_run(prob, X0, nsim, suc_cond, noise, eps, draw):
    """one floor draw of the oracle-driven run: draws 0 and 1 start from the initial states moved
    by one ulp (every nonzero coordinate up, resp. down; exact zeros -- the chasers' initial
    velocities -- stay zero: a signed denormal there is a branch input, not a rounding), draws 2
    and 3 keep the initial states and move every KKT right-hand side by one ulp in every solve
    (two jitter seeds: the backward error of a different summation order, per solve), draws 4
    and 5 run OSQP's KKT solves with every entry's products summed apart before the subtraction
    (two orders of the backward sums, oracle set_solve_order: an implementation of the same solves
    with another valid rounding -- the class of the engine's own remaining difference, its
    blocked / atomic-accumulation triangular solves; everything else it now computes bitwise as
    OSQP, tests/test_gpu_scaling_parity.py)"""
    if draw < 2:
        X = np.where(X0 == 0, X0, np.nextafter(X0, np.inf if draw == 0 else -np.inf))
        return oracle_run(prob, X, nsim, suc_cond, noise, eps)
    if draw < 4:
        return oracle_run(prob, X0, nsim, suc_cond, noise, eps, jitter=draw - 1)
    return oracle_run(prob, X0, nsim, suc_cond, noise, eps, solve_order=draw - 3)


def floor_bound(floors, key, G):
    """lower bound of an agreement figure from the floor's spread over its draws: the worst draw
    less two standard deviations of the draws and one scenario"""
    v = np.array([f[key] for f in floors])
    return float(v.min() - 2 * v.std(ddof=1) - 1.0 / G)
