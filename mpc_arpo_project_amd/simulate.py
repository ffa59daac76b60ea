"""Closed-loop simulators with the reference's call signatures.

`trajectorySimulate(sim_conditions, mpc_params, fail_params, debris)` restates the discrete-time
linear loop of reference src/trajectorySimulate.py:17-388 and `trajectorySimulateC(...)` the
continuous-time nonlinear loop of src/trajectorySimulateC.py:17-446.  The QP assembly comes from
qp_model (bit-identical to the reference's), the per-step reconfiguration is the value-update
restatement of configureDynamicConstraints, the QP solve goes through an OSQP-compatible object
(default: the HIP engine, `osqp_compat.OSQP`), the UKF (noise != None) is the device filter of
`estimation.UnscentedKalmanFilter` and the nonlinear plant is integrated on the device with the
restated scipy RK45 (`estimation.BatchPlant`).  The reference's quirks are kept: Q1 (one-sample
actuation delay; one sub-step in continuous time), Q2 (sequential norm-clip rescale), Q4 (in-track
in-place swap), numpy's global generator seeded with 123 inside trajectorySimulate, the literal
loop start 500 and the float sample test of trajectorySimulateC.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sparse

from .mpcsim import Debris, FailsafeParams, MPCParams, SimConditions, SimRun
from .qp_model import build_problem, configure_dynamic_constraints


def _default_solver():
    from .osqp_compat import OSQP

    return OSQP()


def _terminated(x, rp, rtot, inTrack):
    pos = x[1] if inTrack else x[0]
    return np.linalg.norm(x[0:2]) < rp or pos < rp - rtot


def _select_control(prob, res, xe, xintf, center, side, xr, umax0, lists, i):
    """controller select + clip (src/trajectorySimulate.py:296-319)"""
    impc, ifailsf, ifailsd = lists
    Nx, nx, nu = prob.Nx, prob.nx, prob.nu
    if res.info.status != "solved":
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
    return ctrl, xintf


def _measure(x):
    ymeas = np.empty(2)
    ymeas[0] = np.linalg.norm(x[:2])
    ymeas[1] = math.atan2(x[1], x[0])
    return ymeas


def _update_qp(qp, prob, l, u, xe):
    """QP update after a new estimate (src/trajectorySimulate.py:339-348)"""
    nx, Nx = prob.nx, prob.Nx
    l[:nx] = -xe[:4]
    u[:nx] = -xe[:4]
    qp.update(l=l, u=u)
    Ax, lineq, uineq = configure_dynamic_constraints(prob, xe, swap_in_place=True)
    l[(Nx + 1) * nx:] = lineq
    u[(Nx + 1) * nx:] = uineq
    qp.update(Ax=Ax, l=l, u=u)


def _success(xtruePiece, iterm, xr, distTol, angTol):
    for i in range(iterm - 1, 0, -1):
        dist = np.linalg.norm(xtruePiece[0:2, i] - xr[0:2])
        with np.errstate(divide="ignore", invalid="ignore"):
            ang = abs(math.atan(xtruePiece[3, i] / xtruePiece[2, i])) * (180 / np.pi)
        if dist <= distTol and ang <= angTol:
            return True
    return False


def _ukf(prob, noise, x0, noise_dt=None):
    from .estimation import UnscentedKalmanFilter, observer_model

    Ao, Bou, Qw, R, P0 = observer_model(prob, noise.noise_std, noise_dt)
    return UnscentedKalmanFilter(Ao, Bou, Qw, R, np.hstack([x0, 0., 0.]), P0)


def trajectorySimulate(sim_conditions: SimConditions, mpc_params: MPCParams,
                       fail_params: FailsafeParams, debris: Debris, solver_factory=None):
    np.random.seed(123)  # the reference seeds numpy's global generator (src/...:28)
    noise = sim_conditions.noise
    if noise is not None:
        sigMat = noise.constructSigMat()
        noiseRepeat = noise.noise_length
    else:
        sigMat = np.diag([0., 0., 0., 0.])
        noiseRepeat = 1
    prob = build_problem(sim_conditions, mpc_params, fail_params, debris)
    nx, nu = prob.nx, prob.nu
    T = sim_conditions.time_stp
    nsim = int(sim_conditions.T_final / T)
    rp, rtot = sim_conditions.r_p, sim_conditions.r_tol
    inTrack = sim_conditions.inTrack
    xr = np.asarray(sim_conditions.xr, dtype=float)
    distTol, angTol = sim_conditions.suc_cond
    center = tuple(debris.center) if debris is not None else (-np.inf, -np.inf)
    side = debris.side_length if debris is not None else 0
    Ad_s, Bd_s = sparse.csc_matrix(prob.Ad), sparse.csc_matrix(prob.Bd)

    qp = (solver_factory or _default_solver)()
    l, u = prob.l.copy(), prob.u.copy()
    qp.setup(prob.P, prob.q, prob.A, l, u, warm_start=True, verbose=False)

    x0 = np.asarray(sim_conditions.x0, dtype=float)
    iterm = nsim
    lists = ([], [], [])
    impc, ifailsf, ifailsd = lists
    xtrueP = np.empty([nx, nsim + 1])
    xestO = np.empty([nx + 2, nsim + 1])
    xintf = 0
    noiseStored = np.empty([nx, nsim + 1])
    ctrls = np.empty([nu, nsim + 1])
    ctrls[:, 0] = 0.0
    xtrueP[:, 0] = x0
    xestO[:, 0] = np.hstack([x0, 0., 0.])
    noiseVec = sigMat @ np.random.normal(0, 1, 4)
    noiseStored[:, 0] = noiseVec
    kf = _ukf(prob, noise, x0) if noise is not None else None
    umax0 = prob.umax[0]
    for i in range(nsim):
        if _terminated(xtrueP[:, i], rp, rtot, inTrack):
            iterm = i
            break
        res = qp.solve()
        ctrl, xintf = _select_control(prob, res, xestO[:, i], xintf, center, side, xr, umax0,
                                      lists, i)
        ctrls[:, i + 1] = ctrl
        xtrueP[:, i + 1] = Ad_s @ xtrueP[:, i] + Bd_s @ ctrls[:, i] + noiseVec
        if kf is not None:
            kf.predict(ctrls[:, i])
            kf.update(_measure(xtrueP[:, i + 1]))
            xestO[:, i + 1] = kf.x
        else:
            xestO[:, i + 1] = np.hstack([xtrueP[:, i + 1], [0., 0.]])
        _update_qp(qp, prob, l, u, xestO[:, i + 1])
        if (i + 1) % noiseRepeat == 0:
            noiseVec = sigMat @ np.random.normal(0, 1, 4)
        noiseStored[:, i + 1] = noiseVec

    xtruePiece = np.empty([nx, iterm])
    for idx in lists:
        xtruePiece[:, idx] = xtrueP[:, idx]
    succTraj = _success(xtruePiece, iterm, xr, distTol, angTol)
    controllerSeq = np.empty(iterm)
    controllerSeq[impc] = 1
    controllerSeq[ifailsf] = 2
    controllerSeq[ifailsd] = 3
    return SimRun(iterm, succTraj, xtruePiece, xestO, ctrls, controllerSeq, noiseStored)


def _white_noise(T, Q, dt):
    """python-control white_noise stand-in (the library is absent here; its exact draws are
    unpinned): samples with covariance Q / dt, one column per time in T"""
    Q = np.atleast_2d(Q)
    if not np.any(Q != 0):
        return np.zeros((Q.shape[0], len(T)))
    L = np.linalg.cholesky(Q / dt)
    return L @ np.random.normal(0, 1, (Q.shape[0], len(T)))


def _continuous_append(lists, i):
    """src/simhelpers.py:174-189: carry the controller class through non-sample sub-steps"""
    for lst in lists:
        if lst and lst[-1] == i - 1:
            lst.append(i)
            return


def trajectorySimulateC(sim_conditions: SimConditions, mpc_params: MPCParams,
                        fail_params: FailsafeParams, debris: Debris, solver_factory=None):
    import torch

    from .estimation import BatchPlant

    noise = sim_conditions.noise
    if noise is not None:
        sigMat = noise.constructSigMat()
        noiseRepeat = noise.noise_length
    else:
        sigMat = np.diag([0., 0., 0., 0.])
        noiseRepeat = 1
    prob = build_problem(sim_conditions, mpc_params, fail_params, debris)
    nx, nu, ndi = prob.nx, prob.nu, prob.ndi
    rp, rtot = sim_conditions.r_p, sim_conditions.r_tol
    inTrack = sim_conditions.inTrack
    isDeltaV = sim_conditions.isDeltaV
    n = sim_conditions.mean_mtn
    T = sim_conditions.time_stp
    T_cont = sim_conditions.T_cont
    time_final = sim_conditions.T_final
    nsimD = int(time_final / T)
    nsimC = int(time_final / T_cont)
    xTimeD = np.arange(0, time_final, T)
    xTimeC = np.arange(0, time_final, T_cont)
    xr = np.asarray(sim_conditions.xr, dtype=float)
    distTol, angTol = sim_conditions.suc_cond
    center = tuple(debris.center) if debris is not None else (-np.inf, -np.inf)
    side = debris.side_length if debris is not None else 0
    x0 = np.asarray(sim_conditions.x0, dtype=float)
    hold = int(T / T_cont)

    qp = (solver_factory or _default_solver)()
    l, u = prob.l.copy(), prob.u.copy()
    qp.setup(prob.P, prob.q, prob.A, l, u, warm_start=True, verbose=False)

    iterm = nsimC
    lists = ([], [], [])
    impc, ifailsf, ifailsd = lists
    xtrueP = np.empty([nx, nsimC])
    xestO = np.empty([nx + ndi, nsimD + 1])
    xintf = 0
    noiseStored = np.empty([nx, nsimC])
    ctrls = np.empty([nu, nsimC])
    ctrls[:, :hold + 1] = 0.0
    xtrueP[:, :hold + 1] = x0.reshape(-1, 1)
    xestO[:, 0] = np.hstack([x0, 0., 0.])
    # continuous-time noise (src/trajectorySimulateC.py:295-307)
    Qcont = np.diag([sigMat[0, 0] ** 2, sigMat[0, 0] ** 2])
    noiseInterval = T * noiseRepeat
    noiseTimes = np.arange(0, time_final, noiseInterval)
    noiseIntC = int((noiseRepeat * T) / T_cont)
    V = _white_noise(noiseTimes, Qcont, dt=0.001)
    sum_vec = np.empty([nx, nsimD])
    for j, col in enumerate(V.T):
        noiseStored[:, j * noiseIntC:noiseIntC * (1 + j)] = np.vstack([col.reshape(ndi, 1),
                                                                      np.zeros([2, 1])])
        sum_vec[:, j * noiseRepeat:noiseRepeat * (1 + j)] = \
            hold * np.concatenate([col, np.zeros(2)]).reshape(-1, 1)
    kf = _ukf(prob, noise, x0, noise_dt=T * hold) if noise is not None else None

    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
    plant = BatchPlant(n, 1, device=dev)
    f = dict(dtype=torch.float64, device=plant.device)
    xd = torch.zeros(1, 4, **f)
    ud = torch.zeros(1, 2, **f)
    wd = torch.zeros(1, 4, **f)
    umax0 = prob.umax[0]

    def integrate(i0, cnt, uvec, wvec, t0):
        xd.copy_(torch.as_tensor(xtrueP[:, i0][None]))
        ud.copy_(torch.as_tensor(np.asarray(uvec, dtype=float)[None]))
        wd.copy_(torch.as_tensor(np.asarray(wvec, dtype=float)[None]))
        traj = torch.empty(1, cnt, 4, **f)
        plant.integrate(xd, ud, t0, T_cont, cnt, w=wd, traj=traj)
        return traj[0].cpu().numpy().T

    disc_j = 1
    time = T
    i = 500
    last = 500
    while i < nsimC - 1:
        last = i
        if _terminated(xtrueP[:, i], rp, rtot, inTrack):
            iterm = i
            break
        if (disc_j < nsimD) and (xTimeC[i] == xTimeD[disc_j]):
            res = qp.solve()
            ctrl, xintf = _select_control(prob, res, xestO[:, disc_j - 1], xintf, center, side,
                                          xr, umax0, lists, i)
            ctrls[:, i + 1] = ctrl
            if not isDeltaV:
                xtrueP[:, i + 1] = integrate(i, 1, ctrls[:, i], noiseStored[:, i], time)[:, 0]
            else:  # impulse at the sample; noise rows 2:4 are zero, so the order of adds is moot
                w = noiseStored[:, i] + np.hstack([np.zeros(2), ctrls[:, i]])
                xtrueP[:, i + 1] = integrate(i, 1, np.zeros(nu), w, time)[:, 0]
            if kf is not None:
                kf.predict(ctrls[:, i])
                kf.update(_measure(xtrueP[:, i + 1]))
                xestO[:, disc_j] = kf.x
            else:
                xestO[:, disc_j] = np.hstack([xtrueP[:, i + 1], [0., 0.]])
            _update_qp(qp, prob, l, u, xestO[:, disc_j])
            disc_j = disc_j + 1
            time = time + T_cont
            i += 1
            continue
        # a run of non-sample sub-steps up to the next sample (or the end), split where the
        # stored noise changes; the control is held (ctrls[:, k+1] = ctrls[:, k])
        j = i + 1
        while j < nsimC - 1 and not ((disc_j < nsimD) and (xTimeC[j] == xTimeD[disc_j])) and \
                np.array_equal(noiseStored[:, j], noiseStored[:, i]):
            j += 1
        cnt = j - i
        ctrls[:, i + 1:j + 1] = ctrls[:, i].reshape(-1, 1)
        uh = np.zeros(nu) if isDeltaV else ctrls[:, i]
        xtrueP[:, i + 1:j + 1] = integrate(i, cnt, uh, noiseStored[:, i], time)
        stop = None
        for k in range(i, j):
            if k > i and _terminated(xtrueP[:, k], rp, rtot, inTrack):
                stop = k
                break
            _continuous_append(lists, k)
            time = time + T_cont
        if stop is not None:
            iterm = stop
            last = stop
            break
        i = j
        last = j - 1
    _continuous_append(lists, last + 1)

    xtruePiece = np.empty([nx, iterm])
    xtruePiece[:, :hold + 1] = xtrueP[:, :hold + 1]
    for idx in lists:
        xtruePiece[:, idx] = xtrueP[:, idx]
    succTraj = _success(xtruePiece, iterm, xr, distTol, angTol)
    controllerSeq = np.empty(iterm)
    controllerSeq[:hold] = 0
    controllerSeq[impc] = 1
    controllerSeq[ifailsf] = 2
    controllerSeq[ifailsd] = 3
    controllerSeq[-1] = controllerSeq[-2]
    return SimRun(iterm, succTraj, xtruePiece, xestO, ctrls, controllerSeq, sum_vec)
