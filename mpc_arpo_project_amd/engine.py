"""Batched torch front-end of the HIP engine.

`BatchQP` owns one `mpcqp_handle`: B instances that share the sparsity of P and A (and the values
of P and q) -- the shape of every MPC-QP the reference builds for one scenario family
(reference src/trajectorySimulate.py:216-236).  All tensors are float64 / int32 on the GPU; the
engine never silently moves work to the CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from ._lib import MPCQPError, check

OSQP_INFTY = 1e30
MPCQP_UNSOLVED = -10  # OSQP 0.6 status_val of an instance no solve has touched (include/mpcqp.h)


def _require_gpu(device):
    if not torch.cuda.is_available():
        raise MPCQPError("the MPC-QP engine needs a ROCm GPU (torch.cuda.is_available() is False)")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise MPCQPError(f"device must be a GPU, got {dev}")
    return dev


def triu_csc(P) -> sp.csc_matrix:
    """Upper triangle of P in sorted CSC (what OSQP's Python wrapper hands to the C core)."""
    P = sp.csc_matrix(P)
    if sp.tril(P, -1).nnz:
        P = sp.triu(P, format="csc")
    P = sp.csc_matrix(P)
    P.sort_indices()
    return P


def sorted_csc(A) -> sp.csc_matrix:
    A = sp.csc_matrix(A)
    A.sort_indices()
    return A


@dataclass
class SolveResult:
    x: torch.Tensor         # [B, n] unscaled primal (NaN without solution)
    y: torch.Tensor         # [B, m] unscaled dual
    status: torch.Tensor    # [B] int32, OSQP status_val
    iter: torch.Tensor      # [B] int32
    rho_updates: torch.Tensor
    obj_val: torch.Tensor
    pri_res: torch.Tensor
    dua_res: torch.Tensor
    rho: torch.Tensor


class BatchQP:
    """B OSQP problems with a shared pattern, solved together on one GPU."""

    def __init__(self, P, A, batch: int, device="cuda", stream=None, **settings):
        self.device = _require_gpu(device)
        self.P = triu_csc(P)
        self.A = sorted_csc(A)
        self.n, self.m = self.P.shape[0], self.A.shape[0]
        if self.A.shape[1] != self.n:
            raise ValueError("A must have n columns")
        self.B = int(batch)
        self.settings = _lib.default_settings(**settings)
        self._Pp = np.ascontiguousarray(self.P.indptr, dtype=np.int32)
        self._Pi = np.ascontiguousarray(self.P.indices, dtype=np.int32)
        self._Ap = np.ascontiguousarray(self.A.indptr, dtype=np.int32)
        self._Ai = np.ascontiguousarray(self.A.indices, dtype=np.int32)
        st = _lib.Structure(self.n, self.m,
                            self._Pp.ctypes.data_as(C.POINTER(C.c_int32)),
                            self._Pi.ctypes.data_as(C.POINTER(C.c_int32)),
                            self._Ap.ctypes.data_as(C.POINTER(C.c_int32)),
                            self._Ai.ctypes.data_as(C.POINTER(C.c_int32)))
        with torch.cuda.device(self.device):
            self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
            h = C.c_void_p()
            check(_lib.lib().mpcqp_create(C.byref(st), C.byref(self.settings), self.B,
                                          C.c_void_p(self.stream.cuda_stream), C.byref(h)),
                  "mpcqp_create")
        self._h = h
        self.nnzP = int(self.P.nnz)
        self.nnzA = int(self.A.nnz)
        self._has_data = False
        self._out = None

    # -------------------------------------------------------------------------------- helpers
    def _t(self, a, shape, name):
        t = torch.as_tensor(a, dtype=torch.float64, device=self.device)
        if tuple(t.shape) != tuple(shape):
            t = t.reshape(shape) if t.numel() == int(np.prod(shape)) else None
        if t is None:
            raise ValueError(f"{name} must have shape {shape}")
        return t.contiguous()

    def _batch_vec(self, a, width, name):
        t = torch.as_tensor(a, dtype=torch.float64, device=self.device)
        if t.dim() == 1:
            if t.numel() != width:
                raise ValueError(f"{name} must have {width} entries per instance")
            t = t.unsqueeze(0).expand(self.B, width)
        if tuple(t.shape) != (self.B, width):
            raise ValueError(f"{name} must have shape ({self.B}, {width})")
        return t.contiguous()

    def _keep(self, **tensors):
        # keep the caller-independent copies alive until the stream has consumed them
        self._inflight = tensors

    # ------------------------------------------------------------------------------------ API
    def set_data(self, Px=None, q=None, Ax=None, l=None, u=None):
        Px = self._t(self.P.data if Px is None else Px, (self.nnzP,), "Px")
        q = self._t(q, (self.n,), "q")
        Ax = self._batch_vec(self.A.data if Ax is None else Ax, self.nnzA, "Ax")
        l = self._batch_vec(l, self.m, "l")
        u = self._batch_vec(u, self.m, "u")
        if bool((l > u).any()):
            raise ValueError("lower bound must be lower than or equal to upper bound")
        check(_lib.lib().mpcqp_set_data(self._h, Px.data_ptr(), q.data_ptr(), Ax.data_ptr(),
                                        l.data_ptr(), u.data_ptr()), "mpcqp_set_data")
        self._keep(Px=Px, q=q, Ax=Ax, l=l, u=u)
        self._has_data = True

    def update(self, q=None, l=None, u=None, Ax=None):
        keep = {}
        if q is not None:
            q = self._t(q, (self.n,), "q")
            check(_lib.lib().mpcqp_update_lin_cost(self._h, q.data_ptr()), "mpcqp_update_lin_cost")
            keep["q"] = q
        if l is not None or u is not None:
            if l is None or u is None:
                raise ValueError("update l and u together")
            l = self._batch_vec(l, self.m, "l")
            u = self._batch_vec(u, self.m, "u")
            if bool((l > u).any()):
                raise ValueError("lower bound must be lower than or equal to upper bound")
            check(_lib.lib().mpcqp_update_bounds(self._h, l.data_ptr(), u.data_ptr()),
                  "mpcqp_update_bounds")
            keep.update(l=l, u=u)
        if Ax is not None:
            Ax = self._batch_vec(Ax, self.nnzA, "Ax")
            check(_lib.lib().mpcqp_update_A(self._h, Ax.data_ptr()), "mpcqp_update_A")
            keep["Ax"] = Ax
        self._keep(**keep)

    def _on_stream(self, fn, *tensors):
        """run fn (an ABI call that queues copies on the handle's stream) into freshly allocated
        tensors, then order the caller's current stream after it, so the returned tensors are
        safe to use on the current stream whatever stream the handle runs on"""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)  # the allocations happened on the current stream
        fn()
        for t in tensors:
            t.record_stream(self.stream)
        cur.wait_stream(self.stream)
        return tensors

    def copy_data(self):
        """(Ax, l, u) currently held by the handle, as new device tensors (ordered after the
        handle's stream for the caller's current stream)."""
        f = dict(dtype=torch.float64, device=self.device)
        Ax = torch.empty(self.B, self.nnzA, **f)
        l = torch.empty(self.B, self.m, **f)
        u = torch.empty(self.B, self.m, **f)
        return self._on_stream(lambda: check(_lib.lib().mpcqp_copy_data(
            self._h, Ax.data_ptr(), l.data_ptr(), u.data_ptr()), "mpcqp_copy_data"), Ax, l, u)

    def set_skip(self, mask):
        """int32 device tensor [B] (kept alive by the handle) or None: instances with a non-zero
        entry are skipped by every following solve (outputs and warm state unchanged)"""
        if mask is not None:
            if mask.dtype != torch.int32 or tuple(mask.shape) != (self.B,) or \
                    not mask.is_cuda or not mask.is_contiguous():
                raise ValueError(f"skip mask must be a contiguous int32 tensor of shape ({self.B},)")
        check(_lib.lib().mpcqp_set_skip(self._h, None if mask is None else mask.data_ptr()),
              "mpcqp_set_skip")
        self._skip = mask

    def set_order(self, order):
        """int32 device tensor [B] (kept alive by the handle) or None: a permutation of the
        instance ids, the order in which the persistent launch takes instances (results unchanged;
        mpcqp_set_order).  The tensor is read at every solve, so it may be rewritten in place --
        on the handle's stream, and only with another permutation (a duplicate id would let two
        waves solve one instance at once; a missing id would never be solved).  It is checked to
        be a permutation here, once."""
        if order is not None:
            if order.dtype != torch.int32 or tuple(order.shape) != (self.B,) or \
                    not order.is_cuda or not order.is_contiguous():
                raise ValueError(f"order must be a contiguous int32 tensor of shape ({self.B},)")
            with torch.cuda.stream(self.stream):
                ok = torch.equal(torch.sort(order).values,
                                 torch.arange(self.B, dtype=torch.int32, device=order.device))
            if not ok:
                raise ValueError("order must be a permutation of the instance ids 0..B-1")
        check(_lib.lib().mpcqp_set_order(self._h, None if order is None else order.data_ptr()),
              "mpcqp_set_order")
        self._order = order

    def get_state(self):
        """Warm-start state carried to the next solve (scaled xs, zs, ys; rho; has_state), as new
        device tensors -- the white-box hook the oracle's `state()` mirrors."""
        f = dict(dtype=torch.float64, device=self.device)
        xs = torch.empty(self.B, self.n, **f)
        zs = torch.empty(self.B, self.m, **f)
        ys = torch.empty(self.B, self.m, **f)
        rho = torch.empty(self.B, **f)
        hs = torch.empty(self.B, dtype=torch.int32, device=self.device)
        self._on_stream(lambda: check(_lib.lib().mpcqp_get_state(
            self._h, xs.data_ptr(), zs.data_ptr(), ys.data_ptr(), rho.data_ptr(), hs.data_ptr()),
            "mpcqp_get_state"), xs, zs, ys, rho, hs)
        return dict(x=xs, z=zs, y=ys, rho=rho, has_state=hs)

    def get_scaling(self):
        """The data scaling carried between solves (mpcqp_get_scaling): E of the last solve [B, m]
        and the unscaled P values [B, nnzP] / q [B, n] the next warm solve rescales (OSQP 0.6's
        unscale_data), as new device tensors -- the white-box hook of the oracle's state()/data()"""
        f = dict(dtype=torch.float64, device=self.device)
        E = torch.empty(self.B, self.m, **f)
        Pu = torch.empty(self.B, self.nnzP, **f)
        qu = torch.empty(self.B, self.n, **f)
        self._on_stream(lambda: check(_lib.lib().mpcqp_get_scaling(
            self._h, E.data_ptr(), Pu.data_ptr(), qu.data_ptr()), "mpcqp_get_scaling"), E, Pu, qu)
        return dict(E=E, Pu=Pu, qu=qu)

    def set_state(self, x, z, y, rho, has_state):
        """Overwrite the warm-start state (the reverse of get_state; white-box tests)."""
        f = dict(dtype=torch.float64, device=self.device)
        t = [torch.as_tensor(a, **f).contiguous() for a in (x, z, y, rho)]
        hs = torch.as_tensor(has_state, dtype=torch.int32, device=self.device).contiguous()
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        check(_lib.lib().mpcqp_set_state(self._h, *(a.data_ptr() for a in t), hs.data_ptr()),
              "mpcqp_set_state")
        self._keep(state=(t, hs))

    def warm_start(self, x, y):
        x = self._batch_vec(x, self.n, "x")
        y = self._batch_vec(y, self.m, "y")
        check(_lib.lib().mpcqp_warm_start(self._h, x.data_ptr(), y.data_ptr()), "mpcqp_warm_start")

    def new_result(self) -> SolveResult:
        """Output buffers for solve_async(out=...).  An instance that a skip mask keeps from
        being solved keeps its previous outputs, so a fresh buffer starts from defined values:
        status MPCQP_UNSOLVED (-10, OSQP's 'unsolved'), iter 0, x / y / obj / residuals NaN."""
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            nan = float("nan")
            f = dict(dtype=torch.float64, device=self.device)
            i = dict(dtype=torch.int32, device=self.device)
            return SolveResult(
                x=torch.full((self.B, self.n), nan, **f), y=torch.full((self.B, self.m), nan, **f),
                status=torch.full((self.B,), MPCQP_UNSOLVED, **i), iter=torch.zeros(self.B, **i),
                rho_updates=torch.zeros(self.B, **i), obj_val=torch.full((self.B,), nan, **f),
                pri_res=torch.full((self.B,), nan, **f), dua_res=torch.full((self.B,), nan, **f),
                rho=torch.full((self.B,), nan, **f))

    def _outputs(self):
        if self._out is None:
            self._out = self.new_result()
        return self._out

    def solve_async(self, out: SolveResult = None) -> SolveResult:
        """Enqueue one solve of every instance on the handle's stream (no host sync)."""
        if not self._has_data:
            raise MPCQPError("solve before set_data")
        o = out if out is not None else self._outputs()
        info = _lib.Info(o.status.data_ptr(), o.iter.data_ptr(), o.rho_updates.data_ptr(),
                         o.obj_val.data_ptr(), o.pri_res.data_ptr(), o.dua_res.data_ptr(),
                         o.rho.data_ptr())
        check(_lib.lib().mpcqp_solve(self._h, o.x.data_ptr(), o.y.data_ptr(), C.byref(info)),
              "mpcqp_solve")
        return o

    def solve(self) -> SolveResult:
        o = self.solve_async()
        self.stream.synchronize()
        return o

    def schedule_info(self):
        v = [C.c_int32() for _ in range(5)]
        check(_lib.lib().mpcqp_schedule_info(self._h, *[C.byref(x) for x in v]),
              "mpcqp_schedule_info")
        k, at = C.c_int32(), C.c_int32()
        check(_lib.lib().mpcqp_engine_kind(self._h, C.byref(k)), "mpcqp_engine_kind")
        check(_lib.lib().mpcqp_schedule_kind(self._h, C.byref(at)), "mpcqp_schedule_kind")
        w = [C.c_int32() for _ in range(4)]
        check(_lib.lib().mpcqp_kernel_info(self._h, *[C.byref(x) for x in w]), "mpcqp_kernel_info")
        return dict(engine="kkt", fac_steps=v[0].value,
                    fwd_steps=v[1].value, bwd_steps=v[2].value, lds_bytes=v[3].value,
                    waves_per_cu=v[4].value, atomics_per_step=at.value,
                    waves_per_instance=w[0].value, instances_per_cu=w[1].value,
                    kernel_regs=w[2].value, kernel_scratch_bytes=w[3].value)

    def dims(self):
        v = [C.c_int32() for _ in range(5)]
        check(_lib.lib().mpcqp_dims(self._h, *[C.byref(x) for x in v]), "mpcqp_dims")
        return dict(n=v[0].value, m=v[1].value, nnzP=v[2].value, nnzA=v[3].value,
                    nnzL=v[4].value)

    def close(self):
        if getattr(self, "_h", None):
            try:
                self.stream.synchronize()
            finally:
                _lib.lib().mpcqp_destroy(self._h)
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def data_buffers(qp: BatchQP):
    """Raw device pointers (ints) of the handle's own Ax / l / u buffers (zero-copy updates)."""
    a, l, u = C.c_void_p(), C.c_void_p(), C.c_void_p()
    check(_lib.lib().mpcqp_data_buffers(qp._h, C.byref(a), C.byref(l), C.byref(u)),
          "mpcqp_data_buffers")
    return a.value, l.value, u.value
