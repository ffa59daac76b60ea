"""Scenario / parameter / telemetry objects of the reference, kept with the same names, constructor
signatures and attribute semantics (reference src/mpcsim.py:13-176) so that callers of
`trajectorySimulate(sim_conditions, mpc_params, fail_params, debris)` switch over unchanged.

Plotting (`figurePlotSave`, reference src/mpcsim.py:179-416) and the VPython animation are outside
this build's scope.
"""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np
from scipy import sparse


class Noise:
    """Additive x/y output noise held for `noise_length` control intervals
    (reference src/mpcsim.py:13-32)."""

    def __init__(self, noise_std: Tuple[float, float], noise_length: float):
        self.noise_std = noise_std
        self.noise_length = noise_length

    def constructSigMat(self):
        return np.diag([self.noise_std[0], self.noise_std[1], 0, 0])


class SimConditions:
    """General simulation conditions (reference src/mpcsim.py:35-73).  `hatch_ofst` is derived from
    `inTrack` exactly as the reference does (90 degrees for in-track approaches)."""

    def __init__(self, x0, xr, r_p: float, los_ang: float, r_tol: float, mean_mtn: float,
                 time_stp: float, isReject: bool, suc_cond: Tuple[float, float],
                 noise: Noise = None, inTrack: bool = False, T_cont: float = float("nan"),
                 T_final: int = 100, isDeltaV: bool = False):
        self.x0 = x0
        self.xr = xr
        self.r_p = r_p
        self.los_ang = los_ang
        self.r_tol = r_tol
        self.hatch_ofst = (inTrack * 90) * (np.pi / 180)
        self.mean_mtn = mean_mtn
        self.time_stp = time_stp
        self.isReject = isReject
        self.suc_cond = suc_cond
        self.noise = noise
        self.inTrack = inTrack
        self.T_cont = T_cont
        self.T_final = T_final
        self.isDeltaV = isDeltaV


class SimRun:
    """Telemetry of one closed-loop run (reference src/mpcsim.py:75-97)."""

    def __init__(self, i_term: int, isSuccess: bool, x_true_pcw, x_est, ctrl_hist, ctrlr_seq,
                 noise_hist):
        self.i_term = i_term
        self.isSuccess = isSuccess
        self.x_true_pcw = x_true_pcw
        self.x_est = x_est
        self.ctrl_hist = ctrl_hist
        self.ctrlr_seq = ctrlr_seq
        self.noise_hist = noise_hist


class Debris:
    """Square debris bounding box (reference src/mpcsim.py:99-123)."""

    def __init__(self, center: Tuple[float, float], side_length: float, detect_distance: float):
        self.center = center
        self.side_length = side_length
        self.detect_distance = detect_distance

    def constructVertArr(self):
        """Vertices in the reference's order: (+,+), (-,+), (-,-), (+,-) half-sides."""
        cx, cy = self.center
        h = self.side_length / 2
        return np.array([[cx + h, cy + h], [cx - h, cy + h], [cx - h, cy - h], [cx + h, cy - h]])


class MPCParams:
    """MPC tuning (reference src/mpcsim.py:127-157), including the `swap_xy` in-track helper that
    exchanges the x/y (and vx/vy) weights."""

    def __init__(self, Q_state, R_input, R_slack, V_ecr, horizons, u_lim: Tuple[float, float],
                 swap_xy: bool = False):
        self.Q_state = Q_state
        self.R_input = R_input
        if swap_xy:
            Qd = Q_state.toarray()
            Rd = R_input.toarray()
            Qd[[0, 1, 2, 3], [0, 1, 2, 3]] = Qd[[1, 0, 3, 2], [1, 0, 3, 2]]
            Rd[[0, 1], [0, 1]] = Rd[[1, 0], [1, 0]]
            self.Q_state = sparse.dia_array(Qd)
            self.R_input = sparse.dia_array(Rd)
        self.R_slack = R_slack
        self.V_ecr = V_ecr
        self.Nx = horizons["Nx"]
        self.Nc = horizons["Nc"]
        self.Nb = horizons["Nb"]
        self.u_lim = u_lim


class FailsafeParams:
    """LQR-failsafe / deadbeat parameters (reference src/mpcsim.py:160-176)."""

    def __init__(self, Q_fail, R_fail, C_int, K_dead):
        self.Q_fail = Q_fail
        self.R_fail = R_fail
        self.C_int = C_int
        self.K_dead = K_dead


__all__ = ["Noise", "SimConditions", "SimRun", "Debris", "MPCParams", "FailsafeParams", "math"]
