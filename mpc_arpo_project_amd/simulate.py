"""Closed-loop simulators with the reference's call signatures.

`trajectorySimulate(sim_conditions, mpc_params, fail_params, debris)` restates the
discrete-time linear loop of reference src/trajectorySimulate.py:17-388 (noise=None path): the
QP assembly comes from qp_model (bit-identical to the reference's), the per-step
reconfiguration is the value-update restatement of configureDynamicConstraints, and the QP solve
goes through an OSQP-compatible object (default: the HIP engine, `osqp_compat.OSQP`).  The
reference's quirks Q1 (one-sample actuation delay), Q2 (sequential norm-clip rescale), Q4
(in-track in-place swap) are kept.  The UKF path (noise != None) needs filterpy, which the
reference imports but this image lacks; it is a SURVEY section 8(f) 'next' row.
"""
from __future__ import annotations

import math

import numpy as np

from .mpcsim import Debris, FailsafeParams, MPCParams, SimConditions, SimRun
from .qp_model import build_problem, configure_dynamic_constraints


def _default_solver():
    from .osqp_compat import OSQP

    return OSQP()


def trajectorySimulate(sim_conditions: SimConditions, mpc_params: MPCParams,
                       fail_params: FailsafeParams, debris: Debris, solver_factory=None):
    if sim_conditions.noise is not None:
        raise NotImplementedError("noise != None needs the UKF (filterpy); see SURVEY.md 8(f)")
    prob = build_problem(sim_conditions, mpc_params, fail_params, debris)
    nx, nu, Nx = prob.nx, prob.nu, prob.Nx
    T = sim_conditions.time_stp
    nsim = int(sim_conditions.T_final / T)
    rp, rtot = sim_conditions.r_p, sim_conditions.r_tol
    inTrack = sim_conditions.inTrack
    xr = np.asarray(sim_conditions.xr, dtype=float)
    distTol, angTol = sim_conditions.suc_cond
    center = tuple(debris.center) if debris is not None else (-np.inf, -np.inf)
    side = debris.side_length if debris is not None else 0
    Ad, Bd = prob.Ad, prob.Bd
    import scipy.sparse as sparse

    Ad_s, Bd_s = sparse.csc_matrix(Ad), sparse.csc_matrix(Bd)

    qp = (solver_factory or _default_solver)()
    l, u = prob.l.copy(), prob.u.copy()
    qp.setup(prob.P, prob.q, prob.A, l, u, warm_start=True, verbose=False)

    x0 = np.asarray(sim_conditions.x0, dtype=float)
    iterm = nsim
    ifailsd, ifailsf, impc = [], [], []
    xtrueP = np.empty([nx, nsim + 1])
    xestO = np.empty([nx + 2, nsim + 1])
    xintf = 0
    noiseStored = np.zeros([nx, nsim + 1])
    ctrls = np.empty([nu, nsim + 1])
    ctrls[:, 0] = 0.0
    xtrueP[:, 0] = x0
    xestO[:, 0] = np.hstack([x0, 0., 0.])
    if inTrack:  # the set-up call of configureDynamicConstraints swapped xest in place (quirk Q4)
        pass  # (the reference passes a fresh hstack there, so xestO[:, 0] is not swapped)
    umax0 = prob.umax[0]
    for i in range(nsim):
        if (not inTrack and (np.linalg.norm(xtrueP[0:2, i]) < rp or xtrueP[0, i] < rp - rtot)) or \
           (inTrack and (np.linalg.norm(xtrueP[0:2, i]) < rp or xtrueP[1, i] < rp - rtot)):
            iterm = i
            break
        res = qp.solve()
        if res.info.status != "solved":
            xe = xestO[:, i]
            if (xe[0] - (center[0] + side / 2) < 0 and xe[0] - (center[0] - side / 2) > 0 and
                    xe[1] < (center[1] + side / 2) and xe[1] > (center[1] - side / 2)):
                ifailsd.append(i)
                xintf = xintf + prob.Crefy @ xe[:4] - (center[1] + side / 2)
                ctrl = -prob.K_total @ xe[:4] - prob.K_i @ xintf
            else:
                ifailsf.append(i)
                xintf = xintf + prob.Crefx @ xe[:4] - xr[0]
                ctrl = -prob.Kpf @ xe[:4] - prob.Kif @ xintf
        else:
            impc.append(i)
            xintf = 0
            ctrl = res.x[(Nx + 1) * nx:(Nx + 1) * nx + nu]
        if np.linalg.norm(ctrl) > umax0:
            ctrl[0] = ctrl[0] * (umax0 / np.linalg.norm(ctrl))
            ctrl[1] = ctrl[1] * (umax0 / np.linalg.norm(ctrl))
        ctrls[:, i + 1] = ctrl
        xtrueP[:, i + 1] = Ad_s @ xtrueP[:, i] + Bd_s @ ctrls[:, i] + noiseStored[:, i]
        xestO[:, i + 1] = np.hstack([xtrueP[:, i + 1], [0., 0.]])
        l[:nx] = -xestO[:4, i + 1]
        u[:nx] = -xestO[:4, i + 1]
        qp.update(l=l, u=u)
        Ax, lineq, uineq = configure_dynamic_constraints(prob, xestO[:, i + 1], swap_in_place=True)
        l[(Nx + 1) * nx:] = lineq
        u[(Nx + 1) * nx:] = uineq
        qp.update(Ax=Ax, l=l, u=u)
        noiseStored[:, i + 1] = noiseStored[:, i]

    xtruePiece = np.empty([nx, iterm])
    for idx in (impc, ifailsf, ifailsd):
        xtruePiece[:, idx] = xtrueP[:, idx]
    succTraj = False
    for i in range(iterm - 1, 0, -1):
        dist = np.linalg.norm(xtruePiece[0:2, i] - xr[0:2])
        with np.errstate(divide="ignore", invalid="ignore"):
            ang = abs(math.atan(xtruePiece[3, i] / xtruePiece[2, i])) * (180 / np.pi)
        if dist <= distTol and ang <= angTol:
            succTraj = True
            break
    controllerSeq = np.empty(iterm)
    controllerSeq[impc] = 1
    controllerSeq[ifailsf] = 2
    controllerSeq[ifailsd] = 3
    return SimRun(iterm, succTraj, xtruePiece, xestO, ctrls, controllerSeq, noiseStored)
