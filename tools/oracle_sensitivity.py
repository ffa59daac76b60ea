"""How far the reference semantics itself (the CPU oracle, OSQP 0.6 restated) moves when its input
is perturbed by one unit in the last place: the floor under any status / iteration agreement an fp64
re-implementation with a different summation order can reach.

The cold bench batches of tests/golden/gen_cold_batch.py (B = 65,536, eps 1e-4) are solved twice
by the oracle: on the fixture data and with every A value moved by one ulp in a seeded random
direction (np.nextafter).  The disagreement between the two oracle runs is compared with the HIP
engine's disagreement with the oracle (tests/test_gpu_scale_parity.py): both come from rounding
that long ADMM runs amplify.

    python tools/oracle_sensitivity.py [threads] > profiles/r02/oracle_sensitivity.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import gen_cold_batch as gcb  # noqa: E402
import oracle as orc  # noqa: E402

FAST = 1000


def perturb_ulp(a, seed):
    rng = np.random.default_rng(seed)
    up = rng.random(a.shape) < 0.5
    return np.where(up, np.nextafter(a, np.inf), np.nextafter(a, -np.inf))


def compare(st_a, it_a, st_b, it_b):
    fast = np.maximum(it_a, it_b) <= FAST
    return {
        "status_agreement": float(np.mean(st_a == st_b)),
        "iteration_agreement": float(np.mean(it_a == it_b)),
        "instances": int(st_a.size),
        "status_flips": int(np.sum(st_a != st_b)),
        "flips_among_fast": int(np.sum((st_a != st_b)[fast])),
        "iteration_diffs_among_fast": int(np.sum((it_a != it_b)[fast])),
        "fast_instances": int(fast.sum()),
        "flips_by_min_iterations": {
            f"<= {k}": int(np.sum((st_a != st_b) & (np.minimum(it_a, it_b) <= k)))
            for k in (500, 1000, 2000, 4000)},
    }


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    out = {"what": __doc__.split("\n\n")[0], "fast_threshold_iters": FAST, "configs": {}}
    for tag in ("n20", "n40dv"):
        fx = np.load(os.path.join(REPO, "tests", "golden", f"cold_b65536_{tag}.npz"), allow_pickle=False)
        prob, X, Ax, l, u = gcb.inputs(tag)
        assert gcb.digest(Ax, l, u) == str(fx["sha256"])
        eps = float(fx["eps"])
        _, _, st, it = orc.batch_solve(prob.P, prob.q, prob.A, perturb_ulp(Ax, 1), l, u,
                                       nthreads=threads, eps_abs=eps, eps_rel=eps)
        so, io = fx["status"].astype(np.int32), fx["iter"].astype(np.int32)
        out["configs"][tag] = {"oracle_vs_oracle_1ulp": compare(so, io, st, it)}
        print(tag, out["configs"][tag], file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
