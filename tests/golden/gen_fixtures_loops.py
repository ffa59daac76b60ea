"""Generates tests/golden/cl_noise_n20.npz, clc_n20.npz, clc_n40dv.npz, cl_intrack_n40.npz.  CONTAINER-ONLY: needs
/root/reference (never on the GPU box).

The reference's OWN closed-loop functions run unmodified; the third-party modules it imports
but which are absent from this image are replaced (as in gen_fixtures.py):
  - `osqp`     -> a recorder around the oracle (OSQP 0.6 restatement),
  - `filterpy` -> the oracle's restatement of filterpy 1.4.5's UKF (oracle/estimation_oracle.py),
                  recording every predict / update call,
  - `control`  -> restated dlqr(integral_action) / acker; white_noise only for a zero covariance
                  (the noise=None runs of trajectorySimulateC call it with Q = 0).
  * cl_noise_n20: src.trajectorySimulate.trajectorySimulate with the reference's evaluation noise
    (test/traj_eval_radial.py:23-25: Noise((0.75, 0.75), 50)); the reference seeds numpy's
    global generator itself (src/trajectorySimulate.py:28).
  * clc_n20 / clc_n40dv: src.trajectorySimulateC.trajectorySimulateC, noise=None, T_cont = 1e-3
    (test/traj_eval_radialC.py:38), a 12 s horizon (12,000 solve_ivp sub-steps).
  * cl_intrack_n40 (`python gen_fixtures_loops.py in_track`): trajectorySimulate on the in-track
    approach of test/traj_eval_in_track.py (Nx = 40, swap_xy, noise=None).
Only the resulting arrays are committed; no reference source travels.
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import gen_fixtures as G  # noqa: E402
import estimation_oracle as EO  # noqa: E402  (oracle/ is on sys.path via gen_fixtures)

UKF_LOG = []


class RecordingUKF(EO.UnscentedKalmanFilter):
    def predict(self, dt=None, **kw):
        UKF_LOG.append(dict(x0=self.x.copy(), P0=self.P.copy(), u=np.array(dt, dtype=float)))
        super().predict(dt, **kw)

    def update(self, z, **kw):
        super().update(z, **kw)
        UKF_LOG[-1].update(z=np.array(z, dtype=float), x1=self.x.copy(), P1=self.P.copy())


def install_stubs():
    G.install_stubs()
    m_fpk = sys.modules["filterpy.kalman"]
    m_fpk.UnscentedKalmanFilter = RecordingUKF
    m_fpk.MerweScaledSigmaPoints = EO.MerweScaledSigmaPoints

    def white_noise(T, Q, dt=0):
        Q = np.atleast_2d(Q)
        if np.any(Q != 0):
            raise NotImplementedError("python-control white_noise is not restated")
        return np.zeros((Q.shape[0], len(T)))

    sys.modules["control"].white_noise = white_noise


def run_record(fn, sim, mpc, fail, deb):
    UKF_LOG.clear()
    run = fn(sim, mpc, fail, deb)
    su, steps, solves = G.RECORD["setup"], G.RECORD["steps"], G.RECORD["solves"]
    ups = [s for s in steps if "Ax" in s]
    d = dict(
        step_Ax=np.array([s["Ax"] for s in ups]), step_l=np.array([s["l"] for s in ups]),
        step_u=np.array([s["u"] for s in ups]),
        solve_x=np.array([s["x"] for s in solves]),
        solve_status=np.array([s["status"] for s in solves], dtype=np.int32),
        solve_iter=np.array([s["iter"] for s in solves], dtype=np.int32),
        setup_l=su["l"], setup_u=su["u"], A_data=su["A"].data,
        i_term=np.array(run.i_term), isSuccess=np.array(run.isSuccess),
        x_true_pcw=run.x_true_pcw, ctrlr_seq=run.ctrlr_seq,
    )
    return run, d


def ref_objects_in_track(M, Nx=40):
    """the reference's parameter classes with test/traj_eval_in_track.py's constants (Nx = 40,
    swap_xy = True).  The script omits MPCParams' required u_lim (it would raise a TypeError as
    written); (0.2, 0.2), the radial scripts' value, is supplied."""
    import scipy.sparse as sp

    sim = M.SimConditions(np.array([-10., 100., 0., 0.]), np.array([0., 2.5, 0., 0.]), 2.5,
                          10 * (np.pi / 180), 1.5, 1.107e-3, 0.5, False, (0.2, 45), None, True)
    Q = 8e+02 * sp.diags([0.2 ** 2., 10 ** 2., 3.8 ** 2, 900])
    R = 1000 ** 2 * sp.diags([1, 1])
    Rs = 5 ** 2 * sp.diags([1.5, 1.5, 1, 1, 1e5])
    v = 50000 * np.ones(5)
    v[-2] = -v[-2]
    v[-1] = 1e-09
    mpc = M.MPCParams(Q, R, Rs, v, {"Nx": Nx, "Nc": 5, "Nb": 5}, (0.2, 0.2), swap_xy=True)
    fail = M.FailsafeParams(0.005 * np.diag([0.0001, 1, 100000., 1., 0.01]), 100 * np.diag([1, 1]),
                            np.eye(1, 4), np.zeros([2, 2]))
    deb = M.Debris((0., 40.), 5., 20)
    return sim, mpc, fail, deb


def in_track():
    """cl_intrack_n40: the reference's trajectorySimulate on the in-track approach (noise=None),
    covering the in-track quirk Q4 (src/simhelpers.py:69-75: x/y swapped in the estimate)."""
    install_stubs()
    import src.mpcsim as RM
    from src.trajectorySimulate import trajectorySimulate

    sim, mpc, fail, deb = ref_objects_in_track(RM)
    run, d = run_record(trajectorySimulate, sim, mpc, fail, deb)
    it = int(run.i_term)
    d.update(x_est=run.x_est[:, :it + 1], ctrl_hist=run.ctrl_hist[:, :it + 1])
    np.savez_compressed(os.path.join(HERE, "cl_intrack_n40.npz"), **d)
    print("cl_intrack_n40 i_term", it, "success", run.isSuccess, "solves", len(d["solve_x"]),
          "statuses", np.unique(d["solve_status"], return_counts=True),
          "ctrl", np.unique(run.ctrlr_seq, return_counts=True))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "in_track":
        return in_track()
    install_stubs()
    import src.mpcsim as RM
    from src.trajectorySimulate import trajectorySimulate
    from src.trajectorySimulateC import trajectorySimulateC

    # ---- noisy discrete loop with the UKF
    sim, mpc, fail, deb = G.ref_objects(RM, 20, False)
    sim.noise = RM.Noise((0.75, 0.75), 50)
    run, d = run_record(trajectorySimulate, sim, mpc, fail, deb)
    it = int(run.i_term)
    d.update(x_est=run.x_est[:, :it + 1], ctrl_hist=run.ctrl_hist[:, :it + 1],
             noise=run.noise_hist[:, :it + 1],
             ukf_x0=np.array([r["x0"] for r in UKF_LOG]), ukf_P0=np.array([r["P0"] for r in UKF_LOG]),
             ukf_u=np.array([r["u"] for r in UKF_LOG]), ukf_z=np.array([r["z"] for r in UKF_LOG]),
             ukf_x1=np.array([r["x1"] for r in UKF_LOG]), ukf_P1=np.array([r["P1"] for r in UKF_LOG]))
    np.savez_compressed(os.path.join(HERE, "cl_noise_n20.npz"), **d)
    print("cl_noise_n20 i_term", it, "success", run.isSuccess, "ukf steps", len(UKF_LOG),
          "statuses", np.unique(d["solve_status"], return_counts=True),
          "ctrl", np.unique(run.ctrlr_seq, return_counts=True))

    # ---- continuous-time nonlinear loop (noise=None), short horizon
    for tag, Nx, dv in (("clc_n20", 20, False), ("clc_n40dv", 40, True)):
        sim, mpc, fail, deb = G.ref_objects(RM, Nx, dv)
        sim.T_cont = 0.001
        sim.T_final = 12
        run, d = run_record(trajectorySimulateC, sim, mpc, fail, deb)
        it = int(run.i_term)
        d.update(x_est=run.x_est, ctrl_hist=run.ctrl_hist[:, :it + 1])
        np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **d)
        print(tag, "i_term", it, "success", run.isSuccess, "solves", len(d["solve_x"]),
              "statuses", np.unique(d["solve_status"], return_counts=True),
              "ctrl", np.unique(run.ctrlr_seq, return_counts=True))


if __name__ == "__main__":
    main()
