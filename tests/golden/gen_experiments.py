"""Generates tests/golden/exp_disturb_rej.npz and exp_success_rates.npz.  CONTAINER-ONLY: needs
/root/reference (never on the GPU box).

The reference's two Monte-Carlo experiment scripts, reproduced with the reference's OWN closed-loop
function (src.trajectorySimulate.trajectorySimulate, unmodified) and the same stand-ins as
gen_fixtures_loops.py (osqp -> recorder around the OSQP 0.6 restatement, filterpy -> the UKF
restatement, control -> restated dlqr / acker):
  * test/disturbRejComp.py:56-100: Nx = 40, T_final = 150, Noise((0.7, 0.7), L) for the ten noise
    lengths L, isReject False / True, x0 = (100, 10, 0, 0); final distance
    |x_true_pcw[:, i_term - 1] - xr| and dist_ratio = rej / no-rej per L;
  * test/saved_runs/success_rates_test.py:46-75: Nx = 40, T_final = 300, Noise((0.3, 0.3), 50),
    isReject = True; isSuccess.
trajectorySimulate re-seeds numpy with 123 on every call (src/trajectorySimulate.py:28), so every
Monte-Carlo repetition of one setting is the same run: ONE run per setting is recorded, and the
generator checks that a second call reproduces it bit for bit.  The scripts' outputs follow:
dist_ratios = the per-L ratios of those runs, success_count = 0 or MCnum.

Floor: the same runs with x0 moved by one ulp (components and directions of FLOOR_DRAWS), so the
GPU test can bound the engine's distance from the reference by the reference's own sensitivity
to rounding (the closed loops are chaotic in the solver's rounding, DESIGN.md Parity).
Only the resulting arrays are committed; no reference source travels.

    python tests/golden/gen_experiments.py [--jobs 6]
"""
import argparse
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

NOISE_LENGTHS = (1., 10., 20., 30., 50., 70., 100., 150., 200., 250.)  # disturbRejComp.py:75
X0 = (100., 10., 0., 0.)
XR = np.array([2.5, 0., 0., 0.])
# one-ulp moves of x0: (component, direction); draw 0 is the unperturbed reference run
FLOOR_DRAWS = ((0, +1), (1, -1), (0, -1), (1, +1))


def _x0(draw):
    x0 = np.array(X0)
    if draw > 0:
        c, d = FLOOR_DRAWS[draw - 1]
        x0[c] = np.nextafter(x0[c], np.inf * d)
    return x0


def one_run(job):
    """(experiment, L, isReject, draw) -> the reference's run summary"""
    exp, L, rej, draw = job
    import gen_fixtures_loops as GL

    GL.install_stubs()
    import gen_fixtures as G
    import src.mpcsim as RM
    from src.trajectorySimulate import trajectorySimulate

    sim, mpc, fail, deb = G.ref_objects(RM, 40, False, isReject=rej, x0=tuple(_x0(draw)))
    if exp == "disturb_rej":
        sim.noise, sim.T_final = RM.Noise((0.7, 0.7), L), 150
    else:
        sim.noise, sim.T_final = RM.Noise((0.3, 0.3), 50), 300
    run = trajectorySimulate(sim, mpc, fail, deb)
    it = int(run.i_term)
    out = dict(i_term=it, success=bool(run.isSuccess),
               final_err=float(np.linalg.norm(run.x_true_pcw[:, it - 1] - XR)),
               x_last=run.x_true_pcw[:, it - 1].copy(),
               ctrlr_seq=np.asarray(run.ctrlr_seq, dtype=np.int8),
               statuses=np.array([s["status"] for s in G.RECORD["solves"]], dtype=np.int32),
               noise=run.noise_hist[:, :it + 1].copy())
    if draw == 0 and exp == "disturb_rej" and L == NOISE_LENGTHS[0] and not rej:
        # the Monte-Carlo repetition: a second call must be the same run
        run2 = trajectorySimulate(sim, mpc, fail, deb)
        assert run2.i_term == run.i_term and np.array_equal(run2.x_true_pcw, run.x_true_pcw)
        out["mc_repeat_identical"] = True
    return job, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=6)
    a = ap.parse_args()
    ndraw = 1 + len(FLOOR_DRAWS)
    jobs = [("disturb_rej", L, rej, d) for d in range(ndraw) for L in NOISE_LENGTHS
            for rej in (False, True)]
    jobs += [("success_rates", 50., True, d) for d in range(ndraw)]
    with ProcessPoolExecutor(a.jobs) as ex:
        res = dict(ex.map(one_run, jobs))
    # ---- disturbRejComp
    nL = len(NOISE_LENGTHS)
    shape = (ndraw, nL, 2)
    i_term = np.zeros(shape, np.int32)
    success = np.zeros(shape, bool)
    final_err = np.zeros(shape)
    x_last = np.zeros(shape + (4,))
    for d in range(ndraw):
        for i, L in enumerate(NOISE_LENGTHS):
            for j, rej in enumerate((False, True)):
                r = res[("disturb_rej", L, rej, d)]
                i_term[d, i, j], success[d, i, j] = r["i_term"], r["success"]
                final_err[d, i, j], x_last[d, i, j] = r["final_err"], r["x_last"]
    ref0 = {(L, rej): res[("disturb_rej", L, rej, 0)] for L in NOISE_LENGTHS for rej in (False, True)}
    extra = {}
    for i, L in enumerate(NOISE_LENGTHS):
        for j, rej in enumerate((False, True)):
            r = ref0[(L, rej)]
            extra[f"ctrlr_seq_{i}_{j}"] = r["ctrlr_seq"]
            extra[f"statuses_{i}_{j}"] = r["statuses"]
            extra[f"noise_{i}_{j}"] = r["noise"]
    dist_ratios = final_err[:, :, 1] / final_err[:, :, 0]
    np.savez_compressed(os.path.join(HERE, "exp_disturb_rej.npz"),
                        noise_lengths=np.array(NOISE_LENGTHS), i_term=i_term, success=success,
                        final_err=final_err, x_last=x_last, dist_ratios=dist_ratios,
                        floor_draws=np.array(FLOOR_DRAWS),
                        mc_repeat_identical=np.array(
                            res[("disturb_rej", NOISE_LENGTHS[0], False, 0)]["mc_repeat_identical"]),
                        **extra)
    print("disturb_rej dist_ratios (reference):", np.round(dist_ratios[0], 4).tolist())
    print("  floor draws:", np.round(dist_ratios[1:], 4).tolist())
    print("  i_term", i_term[0].tolist(), "success", success[0].astype(int).tolist())
    # ---- success_rates_test
    sr = [res[("success_rates", 50., True, d)] for d in range(ndraw)]
    np.savez_compressed(os.path.join(HERE, "exp_success_rates.npz"),
                        i_term=np.array([r["i_term"] for r in sr], np.int32),
                        success=np.array([r["success"] for r in sr]),
                        final_err=np.array([r["final_err"] for r in sr]),
                        x_last=np.array([r["x_last"] for r in sr]),
                        ctrlr_seq=sr[0]["ctrlr_seq"], statuses=sr[0]["statuses"],
                        noise=sr[0]["noise"], mc=np.array(300),
                        success_count=np.array(300 * int(sr[0]["success"])))
    print("success_rates: isSuccess", [r["success"] for r in sr], "i_term",
          [r["i_term"] for r in sr], "-> success_count", 300 * int(sr[0]["success"]))


if __name__ == "__main__":
    main()
