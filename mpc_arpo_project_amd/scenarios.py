"""Canonical scenario configurations and the seeded batch generator.

Scenario constants follow the reference's radial experiment script (reference
test/traj_eval_radial.py:17-72) and its in-track sibling (test/traj_eval_in_track.py:14-60); the
horizon is N = Nx = 20 for the headline configuration and 40 for the impulsive-delta-v one.
"""
from __future__ import annotations

import numpy as np
from scipy import sparse

from .mpcsim import Debris, FailsafeParams, MPCParams, Noise, SimConditions

BATCH_SEED = 20250328
LOS_COT = 1.0 / np.tan(10 * np.pi / 180)  # 5.671...


def radial_scenario(Nx: int = 20, Nc: int = 5, Nb: int = 5, isDeltaV: bool = False,
                    isReject: bool = True, noise: Noise = None, x0=(100., 10., 0., 0.),
                    T_final: int = 150, with_debris: bool = True, T_cont: float = float("nan")):
    """(sim_conditions, mpc_params, fail_params, debris) of the radial approach."""
    x0 = np.array(x0, dtype=float)
    xr = np.array([2.5, 0., 0., 0.])
    sim = SimConditions(x0, xr, 2.5, 10 * (np.pi / 180), 1.5, 1.107e-3, 0.5, isReject, (0.2, 45),
                        noise, False, T_cont=T_cont, T_final=T_final, isDeltaV=isDeltaV)
    Q = 8e+02 * sparse.diags([0.2 ** 2., 10 ** 2., 3.8 ** 2, 900])
    R = 1000 ** 2 * sparse.diags([1, 1])
    Rs = 5 ** 2 * sparse.eye(5)
    v_ecr = 50000 * np.ones(5)
    v_ecr[-2] = -1 * v_ecr[-2]
    v_ecr[-1] = 0
    mpc = MPCParams(Q, R, Rs, v_ecr, {"Nx": Nx, "Nc": Nc, "Nb": Nb}, (0.2, 0.2))
    fail = FailsafeParams(0.005 * np.diag([0.0001, 1, 100000., 1., 0.01]), 100 * np.diag([1, 1]),
                          np.eye(1, 4), np.zeros([2, 2]))
    debris = Debris((40., 0.), 5., 20) if with_debris else None
    return sim, mpc, fail, debris


def in_track_scenario(Nx: int = 20, Nc: int = 5, Nb: int = 5, isReject: bool = False,
                      noise: Noise = None, x0=(-10., 100., 0., 0.), T_final: int = 150):
    """In-track approach (reference test/traj_eval_in_track.py); u_lim made explicit (the script
    omits it, which the reference constructor does not allow)."""
    x0 = np.array(x0, dtype=float)
    xr = np.array([0., 2.5, 0., 0.])
    sim = SimConditions(x0, xr, 2.5, 10 * (np.pi / 180), 1.5, 1.107e-3, 0.5, isReject, (0.2, 45),
                        noise, True, T_final=T_final)
    Q = 8e+02 * sparse.diags([0.2 ** 2., 10 ** 2., 3.8 ** 2, 900])
    R = 1000 ** 2 * sparse.diags([1, 1])
    Rs = 5 ** 2 * sparse.diags([1.5, 1.5, 1, 1, 1e5])
    v_ecr = 50000 * np.ones(5)
    v_ecr[-2] = -1 * v_ecr[-2]
    v_ecr[-1] = 1e-09
    mpc = MPCParams(Q, R, Rs, v_ecr, {"Nx": Nx, "Nc": Nc, "Nb": Nb}, (0.2, 0.2), swap_xy=True)
    fail = FailsafeParams(0.005 * np.diag([0.0001, 1, 100000., 1., 0.01]), 100 * np.diag([1, 1]),
                          np.eye(1, 4), np.zeros([2, 2]))
    debris = Debris((0., 40.), 5., 20)
    return sim, mpc, fail, debris


def sample_estimates(B: int, seed: int = BATCH_SEED) -> np.ndarray:
    """Per-instance state/disturbance estimates x_hat = [dx, dy, dvx, dvy, d_x, d_y] (B x 6):
    dx ~ U[20, 110] m, dy ~ U[-15, 15] m rejection-sampled inside the LOS cone
    (dx - 5.671 |dy| >= 1), velocities ~ N(0, 0.05^2) m/s, disturbance estimates ~ N(0, 0.75^2)."""
    rng = np.random.default_rng(seed)
    out = np.empty((B, 6))
    filled = 0
    while filled < B:
        k = max(2 * (B - filled), 64)
        px = rng.uniform(20.0, 110.0, k)
        py = rng.uniform(-15.0, 15.0, k)
        ok = px - LOS_COT * np.abs(py) >= 1.0
        px, py = px[ok], py[ok]
        t = min(B - filled, len(px))
        out[filled:filled + t, 0] = px[:t]
        out[filled:filled + t, 1] = py[:t]
        filled += t
    out[:, 2:4] = rng.normal(0.0, 0.05, (B, 2))
    out[:, 4:6] = rng.normal(0.0, 0.75, (B, 2))
    return out
