"""`OSQP` -- drop-in replacement for the `osqp.OSQP` object on the reference's hot path.

Mirrors the osqp 0.6 Python API exactly as the reference uses it
(reference src/trajectorySimulate.py:242-245 `setup`, :296 `solve`, :342 / :348 `update`;
src/trajectorySimulateC.py:269-272, :338, :399, :405), backed by the HIP engine with batch = 1:

    prob = OSQP()
    prob.setup(P, q, A, l, u, warm_start=True, verbose=False)
    res = prob.solve();  res.x, res.y, res.info.status ('solved', ...), res.info.iter
    prob.update(l=l, u=u);  prob.update(Ax=A.data, l=l, u=u)

Argument meaning and error behaviour follow osqp: dimension mismatches and l > u raise
ValueError; infeasibility / non-convergence are reported through `res.info.status`, never raised.
There is no CPU path: without a GPU or without libmpcqp.so the calls raise MPCQPError.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import scipy.sparse as sp

from ._lib import STATUS
from .engine import BatchQP, sorted_csc, triu_csc

OSQP_INFTY = 1e30


class OSQP:
    def __init__(self, device="cuda"):
        self._device = device
        self._qp = None

    def setup(self, P=None, q=None, A=None, l=None, u=None, **settings):
        if not sp.issparse(P) or not sp.issparse(A):
            raise TypeError("P and A are required to be sparse matrices")
        P = triu_csc(P)
        A = sorted_csc(A)
        n, m = P.shape[0], A.shape[0]
        q = np.asarray(q, dtype=float).reshape(-1)
        if P.shape != (n, n) or A.shape[1] != n or q.shape != (n,):
            raise ValueError("inconsistent problem dimensions")
        l = np.maximum(np.asarray(l, dtype=float).reshape(-1), -OSQP_INFTY)
        u = np.minimum(np.asarray(u, dtype=float).reshape(-1), OSQP_INFTY)
        if l.shape != (m,) or u.shape != (m,):
            raise ValueError("l and u must have length m")
        if np.any(l > u):
            raise ValueError("lower bound must be lower than or equal to upper bound")
        self.n, self.m = n, m
        self._A = A
        self._l, self._u = l.copy(), u.copy()
        self._qp = BatchQP(P, A, batch=1, device=self._device, **settings)
        self._qp.set_data(Px=P.data, q=q, Ax=A.data, l=l, u=u)

    def update(self, q=None, l=None, u=None, Px=None, Px_idx=np.array([]), Ax=None,
               Ax_idx=np.array([])):
        if self._qp is None:
            raise ValueError("setup must be called first")
        if Px is not None:
            raise NotImplementedError("P values are shared by the batch; the reference never updates P")
        if q is not None:
            q = np.asarray(q, dtype=float).reshape(-1)
            if q.shape != (self.n,):
                raise ValueError("q must have length n")
            self._qp.update(q=q)
        if l is not None:
            l = np.maximum(np.asarray(l, dtype=float).reshape(-1), -OSQP_INFTY)
            if l.shape != (self.m,):
                raise ValueError("l must have length m")
        if u is not None:
            u = np.minimum(np.asarray(u, dtype=float).reshape(-1), OSQP_INFTY)
            if u.shape != (self.m,):
                raise ValueError("u must have length m")
        if l is not None or u is not None:
            nl = self._l if l is None else l
            nu = self._u if u is None else u
            if np.any(nl > nu):
                raise ValueError("lower bound must be lower than or equal to upper bound")
            self._l, self._u = nl.copy(), nu.copy()
            self._qp.update(l=nl, u=nu)
        if Ax is not None:
            Ax = np.asarray(Ax, dtype=float).reshape(-1)
            Ax_idx = np.asarray(Ax_idx)
            if len(Ax_idx):
                if len(Ax_idx) != len(Ax):
                    raise ValueError("Ax and Ax_idx must have the same lengths")
                full = self._A.data.copy()
                full[Ax_idx] = Ax
                Ax = full
            if Ax.shape != (self._A.nnz,):
                raise ValueError("Ax must have nnz(A) entries")
            self._A.data[:] = Ax
            self._qp.update(Ax=Ax)

    def warm_start(self, x=None, y=None):
        if x is None or y is None:
            raise NotImplementedError("warm_start needs both x and y in this build")
        self._qp.warm_start(np.asarray(x, dtype=float), np.asarray(y, dtype=float))

    def solve(self):
        r = self._qp.solve()
        st = int(r.status[0])
        info = SimpleNamespace(status=STATUS.get(st, "unknown"), status_val=st, iter=int(r.iter[0]),
                               obj_val=float(r.obj_val[0]), pri_res=float(r.pri_res[0]),
                               dua_res=float(r.dua_res[0]), rho_estimate=float(r.rho[0]),
                               rho_updates=int(r.rho_updates[0]), status_polish=0)
        return SimpleNamespace(x=r.x[0].cpu().numpy(), y=r.y[0].cpu().numpy(), info=info)
