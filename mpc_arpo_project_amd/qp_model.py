"""Construction of the offset-free Clohessy-Wiltshire MPC QP that the reference hands to OSQP.

This is the host-side mirror of the reference's QP assembly, written MI355X-first: the one-time
set-up (discretization, DARE terminal cost, P, q, the dynamics block) uses the same numerical
library calls as the reference so that the matrices are bit-identical, and the per-step
re-configuration (`configureDynamicConstraints`, reference src/simhelpers.py:11-140) is restated as
a *value update in fixed CSC order* instead of a scipy sparse rebuild, in a scalar form (one
scenario) and a vectorised numpy form (a batch of scenarios) whose output feeds the device engine.

Provenance of each piece (all citations into the reference):
  continuous CW model + discretization ....... src/trajectorySimulate.py:72-111
  constraint rows C, input limits, slack map . src/trajectorySimulate.py:132-166
  virtual-LQR terminal cost (DARE) ........... src/trajectorySimulate.py:174-177
  failsafe LQR (integral action), deadbeat ... src/trajectorySimulate.py:179-203
  P, q, Aeq, block matrices, initial l/u ..... src/trajectorySimulate.py:210-236
  dynamics equality block .................... src/simhelpers.py:142-172 (constructOsqpAeq)
  per-step A values and bounds ............... src/simhelpers.py:11-140 (configureDynamicConstraints)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy as sp
import scipy.integrate  # noqa: F401  (sp.integrate.quad)
import scipy.linalg  # noqa: F401
from scipy import sparse

from .mpcsim import Debris, FailsafeParams, MPCParams, SimConditions

# ------------------------------------------------------------------------------------------------
# small linear-systems helpers (restatements of the python-control calls the reference makes;
# python-control is not installed in this image)
# ------------------------------------------------------------------------------------------------


def dlqr_integral(A, B, Q, R, C_int):
    """python-control `dlqr(A, B, Q, R, integral_action=C)` (used at reference
    src/trajectorySimulate.py:185): augment with a discrete integrator x_i+ = x_i + C x, solve the
    DARE and return K = (R + B'SB)^-1 B'SA of the augmented system."""
    A = np.asarray(A, dtype=float)
    B = np.asarray(B, dtype=float)
    C_int = np.atleast_2d(np.asarray(C_int, dtype=float))
    nx, nu = B.shape
    nr = C_int.shape[0]
    Aa = np.block([[A, np.zeros((nx, nr))], [C_int, np.eye(nr)]])
    Ba = np.vstack([B, np.zeros((nr, nu))])
    S = sp.linalg.solve_discrete_are(Aa, Ba, Q, R)
    return np.linalg.solve(Ba.T @ S @ Ba + R, Ba.T @ S @ Aa)


def acker(A, B, poles):
    """python-control `acker` (Ackermann pole placement, reference src/trajectorySimulate.py:198)."""
    A = np.asarray(A, dtype=float)
    B = np.asarray(B, dtype=float)
    n = A.shape[0]
    ctrb = np.hstack([np.linalg.matrix_power(A, i) @ B for i in range(n)])
    if np.linalg.matrix_rank(ctrb) != n:
        raise ValueError("System not reachable; pole placement invalid")
    p = np.real(np.poly(poles))
    npoly = np.size(p)
    pmat = p[npoly - 1] * np.linalg.matrix_power(A, 0)
    for i in np.arange(1, npoly):
        pmat = pmat + p[npoly - i - 1] * np.linalg.matrix_power(A, i)
    K = np.linalg.solve(ctrb, pmat)
    return np.atleast_2d(K[-1][:])


def cw_continuous(n):
    """Planar linear CW model: state [dx, dy, dvx, dvy], acceleration inputs."""
    Ap = np.array([[0., 0., 1., 0.],
                   [0., 0., 0., 1.],
                   [3 * n ** 2, 0., 0., 2 * n],
                   [0., 0., -2 * n, 0.]])
    Bp = np.array([[0., 0.], [0., 0.], [1., 0.], [0., 1.]])
    return Ap, Bp


_EXP_INTEGRAL_CACHE: dict = {}


def expm_integral(Ap, T):
    """Entry-wise int_0^T e^{Ap s} ds exactly as the reference evaluates it: sympy's symbolic
    matrix exponential, lambdified, integrated with scipy quad (src/trajectorySimulate.py:101-107)."""
    key = (Ap.tobytes(), float(T))
    if key not in _EXP_INTEGRAL_CACHE:
        import sympy as sy

        import warnings

        s = sy.symbols("x")
        eAs = (sy.Matrix(Ap) * s).exp()
        out = np.empty(Ap.shape)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", np.exceptions.ComplexWarning)
            for (i, j), fij in np.ndenumerate(eAs):
                out[i, j] = sp.integrate.quad(sy.lambdify((s), fij), 0., T)[0]
        _EXP_INTEGRAL_CACHE[key] = out
    return _EXP_INTEGRAL_CACHE[key].copy()


# ------------------------------------------------------------------------------------------------
# the problem object
# ------------------------------------------------------------------------------------------------


@dataclass
class MPCProblem:
    """Everything the closed loop and the batch engine need about one scenario family."""

    nx: int
    nu: int
    ny: int
    ndi: int
    Nx: int
    Nc: int
    Nb: int
    T: float
    Ad: np.ndarray
    Bd: np.ndarray
    K: np.ndarray
    S: np.ndarray
    C: np.ndarray
    umin: np.ndarray
    umax: np.ndarray
    P: sparse.csc_matrix  # full symmetric, as the reference passes it to OSQP
    q: np.ndarray
    A: sparse.csc_matrix  # structural pattern, values at the set-up state
    l: np.ndarray
    u: np.ndarray
    # position (in A.data, CSC order) of the per-step varying values, per prediction stage k
    pos_c1: np.ndarray = field(default=None)
    pos_c2: np.ndarray = field(default=None)
    pos_slope: np.ndarray = field(default=None)
    # scenario constants used by configureDynamicConstraints
    rp: float = 0.0
    rtol: float = 0.0
    xr: np.ndarray = None
    rx: float = 0.0
    ry: float = 0.0
    isReject: bool = True
    inTrack: bool = False
    has_debris: bool = True
    center: tuple = (0.0, 0.0)
    side: float = 0.0
    detect: float = np.inf
    verts: np.ndarray = None  # debris vertices, already rotated for in-track runs
    # failsafe / deadbeat gains (reference src/trajectorySimulate.py:179-203)
    Kpf: np.ndarray = None
    Kif: np.ndarray = None
    K_total: np.ndarray = None
    K_i: np.ndarray = None
    Crefx: np.ndarray = None
    Crefy: np.ndarray = None

    @property
    def n(self) -> int:
        return self.P.shape[0]

    @property
    def m(self) -> int:
        return self.A.shape[0]

    @property
    def nnzA(self) -> int:
        return self.A.nnz

    @property
    def u0_slice(self) -> slice:
        """where the first control move sits in x (reference src/trajectorySimulate.py:314)"""
        s = (self.Nx + 1) * self.nx
        return slice(s, s + self.nu)


def construct_aeq(Nx, Nc, Ad, Bd, K, ny):
    """Dynamics equality block (reference src/simhelpers.py:142-172): x0 pinned, x_{k+1} = Ad x_k +
    Bd u_k for k < Nc, closed-loop (Ad - Bd K) propagation afterwards, coupling at (Nc+1, Nc)."""
    nx = Ad.shape[0]
    Ad = sparse.csc_matrix(Ad)
    Bd = sparse.csc_matrix(Bd)
    Acl = Ad - Bd @ K
    top = sparse.kron(sparse.eye(Nc + 1), -sparse.eye(nx)) + sparse.kron(sparse.eye(Nc + 1, k=-1), Ad)
    tail = sparse.kron(sparse.eye(Nx - Nc), -sparse.eye(nx)) + sparse.kron(
        sparse.eye(Nx - Nc, k=-1), Acl)
    link = sparse.lil_matrix((Nx + 1, Nx + 1))
    link[Nc + 1, Nc] = 1
    Ax_blk = sparse.block_diag([top, tail], format="csr") + sparse.kron(sparse.csr_matrix(link), Acl)
    sel = sparse.vstack([sparse.csc_matrix((1, Nc)), sparse.eye(Nc), sparse.csc_matrix((Nx - Nc, Nc))])
    Bu = sparse.kron(sel, sparse.hstack([Bd, np.zeros([nx, ny])]))
    return sparse.hstack([Ax_blk, Bu])


def _assemble_A(Aeq, C, blocks, Nx):
    """[[Aeq, AextCol], [kron(I, C), Block12; Block21, Aineq2 | 0], [AextRow]] as CSC with sorted
    indices (the order OSQP stores; reference src/simhelpers.py:109-113)."""
    Aineq2, Block12, Block21, AextRow, AextCol = blocks
    Aineq1 = sparse.kron(sparse.eye(Nx + 1), C)
    Aineq = sparse.block_array(([Aineq1, Block12], [Block21, Aineq2]), format="dia")
    A = sparse.vstack([Aeq, Aineq], format="csc")
    A = sparse.hstack([A, AextCol])
    A = sparse.vstack([A, AextRow])
    A = sparse.csc_matrix(A)
    A.sort_indices()
    return A


def _debris_geometry(sim_conditions: SimConditions, debris: Debris):
    if debris is None:
        return False, (-np.inf, -np.inf), 0.0, np.inf, None
    verts = debris.constructVertArr()
    if sim_conditions.inTrack:
        verts = verts[[1, 2, 3, 0], :]  # bounding box turned on its side (src/simhelpers.py:51-54)
    return True, tuple(debris.center), float(debris.side_length), float(debris.detect_distance), verts


def build_problem(sim_conditions: SimConditions, mpc_params: MPCParams,
                  fail_params: FailsafeParams = None, debris: Debris = None) -> MPCProblem:
    """One-time QP assembly of `trajectorySimulate` (reference src/trajectorySimulate.py:45-245)."""
    n = sim_conditions.mean_mtn
    T = sim_conditions.time_stp
    gam, rp, rtot, phi = (sim_conditions.los_ang, sim_conditions.r_p, sim_conditions.r_tol,
                          sim_conditions.hatch_ofst)
    x0 = np.asarray(sim_conditions.x0, dtype=float)
    xr = np.asarray(sim_conditions.xr, dtype=float)
    has_debris = debris is not None
    center = tuple(debris.center) if has_debris else (-np.inf, -np.inf)
    side = debris.side_length if has_debris else 0

    Ap, Bp = cw_continuous(n)
    nx, nu = Bp.shape
    ndi = 2
    Ad_s = sparse.csc_matrix(sp.linalg.expm(Ap * T))
    if not sim_conditions.isDeltaV:
        Bd_s = sparse.csc_matrix(expm_integral(Ap, T) @ Bp)
    else:
        Bd_s = sparse.csc_matrix(Ad_s @ np.vstack([np.zeros([2, 2]), np.eye(2)]))

    # constraint rows: LOS cone x2, radial floor, velocity 1-norm, debris line
    den = (rp - rtot) * math.sin(gam)
    C11, C12 = math.sin(phi + gam) / den, -math.cos(phi + gam) / den
    C21, C22 = -math.sin(phi - gam) / den, math.cos(phi - gam) / den
    if has_debris:
        verts0 = debris.constructVertArr()
        if x0[0] - (center[0] + side / 2) < 0 and x0[0] - (center[0] - side / 2) > 0:
            slope = (x0[1] - verts0[1, 1]) / (x0[0] - verts0[1, 0])
        else:
            slope = (x0[1] - verts0[0, 1]) / (x0[0] - verts0[0, 0])
    else:
        slope = 0
    C = np.array([[C11, C12, 0., 0.],
                  [C21, C22, 0., 0.],
                  [1., 0., 0., 0.],
                  [0., 0., 1., 1.],
                  [-slope, 1., 0., 0.]])
    if sim_conditions.inTrack:
        C[2, :] = np.array([0., 1., 0., 0.])
    ny = C.shape[0]

    ulim = mpc_params.u_lim
    umin = np.hstack([-ulim[0], -ulim[1], np.zeros(ny)])
    umax = np.hstack([ulim[0], ulim[1], np.inf * np.ones(ny)])
    Dmap = np.hstack([np.zeros([ny, nu]), np.diag(mpc_params.V_ecr)])

    Q, Ru, Rs = mpc_params.Q_state, mpc_params.R_input, mpc_params.R_slack
    R = sparse.block_diag([Ru, Rs])
    S = sp.linalg.solve_discrete_are(Ad_s.toarray(), Bd_s.toarray(), Q.toarray(), Ru.toarray())
    K = np.asarray(np.linalg.inv(Ru + np.transpose(Bd_s) @ S @ Bd_s) @ (np.transpose(Bd_s) @ S @ Ad_s))
    if not np.all(np.linalg.eigvals(S) > 0):
        raise ValueError("Riccati solution not positive definite")

    Nx, Nc, Nb = mpc_params.Nx, mpc_params.Nc, mpc_params.Nb
    P = sparse.block_diag([sparse.kron(sparse.eye(Nx), Q), S, sparse.kron(sparse.eye(Nc), R),
                           1 * sparse.eye(ndi)], format="csc")
    q = np.hstack([np.kron(np.ones(Nx), -Q @ xr), -S @ xr, np.zeros(Nc * (nu + ny)), np.zeros(ndi)])
    Aeq = construct_aeq(Nx, Nc, Ad_s, Bd_s, K, ny)

    Aineq2 = sparse.kron(sparse.eye(Nc), sparse.eye(nu + ny))
    Block12 = sparse.vstack([np.kron(np.eye(Nc), Dmap),
                             np.kron(np.zeros([(Nx + 1) - Nc, Nc]), np.zeros([ny, nu + ny]))])
    Block21 = sparse.coo_matrix((Nc * (nu + ny), (Nx + 1) * nx))
    AextCol = sparse.vstack([np.zeros([nx, ndi]),
                             np.kron(np.ones([Nx, 1]), np.vstack([np.eye(ndi), np.zeros([nx - ndi, ndi])])),
                             np.zeros([(Nx + 1) * ny, ndi]), np.zeros([Nc * (nu + ny), ndi])])
    AextRow = sparse.csc_matrix(np.hstack([np.zeros([ndi, (Nx + 1) * nx]),
                                           np.zeros([ndi, Nc * (nu + ny)]), np.eye(ndi)]))
    blocks = (Aineq2, Block12, Block21, AextRow, AextCol)

    hd, ctr, sd, det, verts = _debris_geometry(sim_conditions, debris)
    prob = MPCProblem(nx=nx, nu=nu, ny=ny, ndi=ndi, Nx=Nx, Nc=Nc, Nb=Nb, T=T,
                      Ad=Ad_s.toarray(), Bd=Bd_s.toarray(), K=K, S=S, C=C, umin=umin, umax=umax,
                      P=P, q=q, A=None, l=None, u=None, rp=rp, rtol=rtot, xr=xr.copy(),
                      rx=float(xr[0]), ry=float(xr[1]),
                      isReject=bool(sim_conditions.isReject), inTrack=bool(sim_conditions.inTrack),
                      has_debris=hd, center=ctr, side=sd, detect=det, verts=verts)

    # A pattern and the CSC positions of the three varying entries per stage: assemble with probe
    # values and diff (C[3,2] = C1, C[3,3] = C2, C[4,0] = -slope in every one of the Nx+1 copies)
    def probe(c1, c2, s):
        Cp = C.copy()
        Cp[3, 2], Cp[3, 3], Cp[4, 0] = c1, c2, s
        return _assemble_A(Aeq, Cp, blocks, Nx)

    base = probe(1.0, 1.0, 0.5)
    for other in (probe(-1.0, 1.0, 0.5), probe(1.0, -1.0, 0.5), probe(1.0, 1.0, 0.25)):
        if other.nnz != base.nnz or not (np.array_equal(other.indices, base.indices)
                                         and np.array_equal(other.indptr, base.indptr)):
            raise RuntimeError("A sparsity pattern is not stable under value changes")
    prob.pos_c1 = np.flatnonzero(probe(-1.0, 1.0, 0.5).data != base.data)
    prob.pos_c2 = np.flatnonzero(probe(1.0, -1.0, 0.5).data != base.data)
    prob.pos_slope = np.flatnonzero(probe(1.0, 1.0, 0.25).data != base.data)
    assert len(prob.pos_c1) == len(prob.pos_c2) == len(prob.pos_slope) == Nx + 1
    prob.A = base
    if not has_debris:
        # the reference's pattern has no debris-line x entries when slope == 0 (no debris)
        keep = np.ones(base.nnz, bool)
        keep[prob.pos_slope] = False
        A0 = probe(1.0, 1.0, 0.0)
        A0.eliminate_zeros()
        prob.A = A0
        prob.pos_c1 = np.flatnonzero(probe(-1.0, 1.0, 0.0).data != probe(1.0, 1.0, 0.0).data)
        prob.pos_c2 = np.flatnonzero(probe(1.0, -1.0, 0.0).data != probe(1.0, 1.0, 0.0).data)
        prob.pos_slope = np.zeros(0, dtype=np.int64)
        _ = keep
    prob._blocks = blocks  # kept for the scipy cross-check in tests
    prob._Aeq = Aeq
    prob._base_data = prob.A.data.copy()

    Ax0, lineq, uineq = configure_dynamic_constraints(prob, np.hstack([x0, 0., 0.]))
    prob.A = sparse.csc_matrix((Ax0, prob.A.indices, prob.A.indptr), shape=prob.A.shape)
    leq = np.hstack([-x0, np.zeros(Nx * nx)])
    prob.l = np.hstack([leq, lineq])
    prob.u = np.hstack([leq, uineq])

    if fail_params is not None:
        Crefx = np.atleast_2d(fail_params.C_int)
        Kf = dlqr_integral(prob.Ad, prob.Bd, fail_params.Q_fail, fail_params.R_fail, Crefx)
        nr = Crefx.shape[0]
        prob.Kpf, prob.Kif, prob.Crefx = Kf[:, :nx], Kf[:, nx:nx + nr], Crefx
        prob.Crefy = np.array([[0., 1., 0., 0.]])
        Bd_prune = prob.Bd[:, 1].reshape(nx, 1)[[1, 3], :]
        Ad_prune = prob.Ad[[1, 3], :][:, [1, 3]]
        A_aug = np.block([[Ad_prune, np.zeros([2, 1])], [np.array([[1, 0]]), np.eye(1)]])
        B_aug = np.block([[Bd_prune], [np.zeros([1, 1])]])
        K_prune = acker(A_aug, B_aug, np.array([0, 0, 0]))
        K_total = np.zeros([nu, nx])
        K_total[1, 1] = K_prune[0, 0]
        K_total[1, 3] = K_prune[0, 1]
        prob.K_total = K_total
        prob.K_i = np.vstack([0, K_prune[0, 2]])
    return prob


# ------------------------------------------------------------------------------------------------
# per-step reconfiguration (reference src/simhelpers.py:11-140)
# ------------------------------------------------------------------------------------------------


def _region(prob: MPCProblem, xe0, xe1, xc0, xc1):
    """Debris-line slope/intercept and the state bounds of one stage (scalar restatement).
    xe*: estimate after the in-track swap (used for the region tests), xc*: unswapped estimate
    (used for the line through the vertex), as in the reference."""
    cx, cy = prob.center
    if prob.inTrack:
        cx, cy = cy, cx
    h = prob.side / 2
    inside = (xe0 - (cx + h) < 0) and (xe0 - (cx - h) > 0)
    near = (xe0 - (cx + h) < prob.detect) and (xe0 - (cx + h) > 0)
    slope, inter = 0.0, None
    V = prob.verts
    if xe1 >= 0:
        if inside:
            vx, vy = V[1, 0], V[1, 1]
        elif prob.has_debris:
            vx, vy = V[0, 0], V[0, 1]
        else:
            vx = None
    else:
        if inside:
            vx, vy = V[2, 0], V[2, 1]
        elif prob.has_debris:
            vx, vy = V[3, 0], V[3, 1]
        else:
            vx = None
    if vx is not None:
        slope = (xc1 - vy) / (xc0 - vx)
        inter = -slope * xc0 + xc1
    l1 = np.absolute(xc0 - prob.rx) + np.absolute(xc1 - prob.ry)
    if xe1 >= 0:
        lo5 = inter if (inside or near) else -np.inf
        xmin = np.array([1., 1., prob.rp, 0., lo5])
        xmax = np.array([np.inf, np.inf, np.inf, l1, np.inf])
    else:
        hi5 = inter if (inside or near) else np.inf
        xmin = np.array([1., 1., prob.rp, 0., -np.inf])
        xmax = np.array([np.inf, np.inf, np.inf, l1, hi5])
    return slope, xmin, xmax


def configure_dynamic_constraints(prob: MPCProblem, xest, swap_in_place: bool = False):
    """Scalar restatement of configureDynamicConstraints for ONE scenario.

    Returns (Ax values in CSC order, lineq, uineq).  With `swap_in_place` the in-track quirk Q4 is
    reproduced: `xest[0], xest[1]` are swapped in the caller's array (src/simhelpers.py:72)."""
    xest = np.asarray(xest)
    C1 = (-1, 1)[bool(xest[2] >= 0)]
    C2 = (-1, 1)[bool(xest[3] >= 0)]
    xc0, xc1 = float(xest[0]), float(xest[1])
    if prob.inTrack:
        xe0, xe1 = xc1, xc0
        if swap_in_place:
            xest[0], xest[1] = xest[1], xest[0]
    else:
        xe0, xe1 = xc0, xc1
    slope, xmin, xmax = _region(prob, xe0, xe1, xc0, xc1)
    Ax = prob._base_data.copy()
    Ax[prob.pos_c1] = C1
    Ax[prob.pos_c2] = C2
    if len(prob.pos_slope):
        Ax[prob.pos_slope] = -slope
    Nx, Nb, Nc, ny = prob.Nx, prob.Nb, prob.Nc, prob.ny
    d = prob.isReject * np.asarray(xest[4:6], dtype=float)
    lineq = np.hstack([np.kron(np.ones(Nb + 1), xmin), np.kron(np.ones(Nx - Nb), -np.inf * np.ones(ny)),
                       np.kron(np.ones(Nc), prob.umin), d])
    uineq = np.hstack([np.kron(np.ones(Nb + 1), xmax), np.kron(np.ones(Nx - Nb), np.inf * np.ones(ny)),
                       np.kron(np.ones(Nc), prob.umax), d])
    return Ax, lineq, uineq


def full_bounds(prob: MPCProblem, xest, lineq, uineq):
    """l/u of the whole QP: dynamics rows pinned to -x_hat, then the reconfigured rows
    (reference src/trajectorySimulate.py:340-347)."""
    nx, Nx = prob.nx, prob.Nx
    eq = np.zeros((Nx + 1) * nx)
    eq[:nx] = -np.asarray(xest[:nx], dtype=float)
    return np.hstack([eq, lineq]), np.hstack([eq, uineq])


def configure_batch(prob: MPCProblem, xest_batch):
    """Vectorised configureDynamicConstraints + bound assembly for a batch of estimates
    (B x 6: [x, y, vx, vy, dx, dy]).  Returns Ax (B, nnzA), l (B, m), u (B, m), all float64;
    identical, value for value, to calling the scalar version per row."""
    X = np.asarray(xest_batch, dtype=float)
    B = X.shape[0]
    xc0, xc1 = X[:, 0], X[:, 1]
    if prob.inTrack:
        xe0, xe1 = xc1, xc0
    else:
        xe0, xe1 = xc0, xc1
    C1 = np.where(X[:, 2] >= 0, 1.0, -1.0)
    C2 = np.where(X[:, 3] >= 0, 1.0, -1.0)
    cx, cy = prob.center
    if prob.inTrack:
        cx, cy = cy, cx
    h = prob.side / 2
    with np.errstate(invalid="ignore", divide="ignore"):
        inside = ((xe0 - (cx + h)) < 0) & ((xe0 - (cx - h)) > 0)
        near = ((xe0 - (cx + h)) < prob.detect) & ((xe0 - (cx + h)) > 0)
        up = xe1 >= 0
        if prob.has_debris:
            V = prob.verts
            vx = np.where(up, np.where(inside, V[1, 0], V[0, 0]), np.where(inside, V[2, 0], V[3, 0]))
            vy = np.where(up, np.where(inside, V[1, 1], V[0, 1]), np.where(inside, V[2, 1], V[3, 1]))
            slope = (xc1 - vy) / (xc0 - vx)
            inter = -slope * xc0 + xc1
        else:
            slope = np.zeros(B)
            inter = np.full(B, np.nan)
        l1 = np.absolute(xc0 - prob.rx) + np.absolute(xc1 - prob.ry)
    act = inside | near
    lo5 = np.where(up & act, inter, -np.inf)
    hi5 = np.where(~up & act, inter, np.inf)
    Nx, Nb, Nc, ny, nx = prob.Nx, prob.Nb, prob.Nc, prob.ny, prob.nx
    Ax = np.broadcast_to(prob._base_data, (B, prob.nnzA)).copy()
    Ax[:, prob.pos_c1] = C1[:, None]
    Ax[:, prob.pos_c2] = C2[:, None]
    if len(prob.pos_slope):
        Ax[:, prob.pos_slope] = -slope[:, None]
    m = prob.m
    l = np.zeros((B, m))
    u = np.zeros((B, m))
    l[:, :nx] = -X[:, :nx]
    u[:, :nx] = -X[:, :nx]
    r0 = (Nx + 1) * nx
    xmin = np.empty((B, ny))
    xmax = np.empty((B, ny))
    xmin[:, 0], xmin[:, 1], xmin[:, 2], xmin[:, 3], xmin[:, 4] = 1., 1., prob.rp, 0., lo5
    xmax[:, 0], xmax[:, 1], xmax[:, 2], xmax[:, 3], xmax[:, 4] = np.inf, np.inf, np.inf, l1, hi5
    for k in range(Nb + 1):
        l[:, r0 + k * ny:r0 + (k + 1) * ny] = xmin
        u[:, r0 + k * ny:r0 + (k + 1) * ny] = xmax
    r1 = r0 + (Nb + 1) * ny
    r2 = r0 + (Nx + 1) * ny
    l[:, r1:r2] = -np.inf
    u[:, r1:r2] = np.inf
    w = prob.nu + ny
    for k in range(Nc):
        l[:, r2 + k * w:r2 + (k + 1) * w] = prob.umin
        u[:, r2 + k * w:r2 + (k + 1) * w] = prob.umax
    r3 = r2 + Nc * w
    d = prob.isReject * X[:, 4:6]
    l[:, r3:r3 + prob.ndi] = d
    u[:, r3:r3 + prob.ndi] = d
    return Ax, l, u
