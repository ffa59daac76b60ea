"""The full-length sweep parity at a larger sample than the GPU test (tests/test_gpu_sweep_parity.py
runs 256 scenarios, where one standard error of a same-run share is ~0.03): the oracle-driven run,
all six one-ulp floor draws of sweep_parity.floor_run and the engine-driven run of one case, each
compared with the oracle run.  Prints one JSON object (the figures, the draws' mean / sd and where
the engine sits in units of the draws' sd and of the binomial standard error).

    python tools/parity_floor.py [--case radial20] [--n 1024] > profiles/r05/evidence/parity_floor_radial20.json
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

import sweep_parity as spp  # noqa: E402
from mpc_arpo_project_amd import sweep  # noqa: E402

CASES = {
    "radial20": ("radial", 20, (0.3, 0.3, 50), True, 150.0),
    "radial40": ("radial", 40, (0.75, 0.75, 50), True, 150.0),
    "in_track40": ("in_track", 40, None, False, 150.0),
}
KEYS = ("same_run", "i_term_agree", "success_agree")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="radial20", choices=sorted(CASES))
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--hybrid-only", action="store_true",
                    help="the oracle run, the engine run and the two hybrid runs only (no floor draws)")
    a = ap.parse_args()
    scen, nx, noise, rej, tf = CASES[a.case]
    sim, prob = sweep.build(scen, nx, noise, rej, tf)
    nsim = int(sim.T_final / sim.time_stp)
    X0 = sweep.initial_conditions(scen, a.n)
    t0 = time.time()
    orc = spp.oracle_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3)
    print(f"oracle run: {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    eng = spp.compare(spp.engine_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3), orc)
    print(f"engine: {time.time() - t0:.1f} s {eng['same_run']}", file=sys.stderr, flush=True)
    # the hybrid runs (round 6): the oracle with the engine's KKT factorization and blocked solves
    # (1), and with the engine's fused ADMM updates as well (2: the engine's arithmetic, bitwise --
    # tests/test_gpu_hybrid.py); which of the two differences moves the loops
    hyb = {}
    for h in (1, 2):
        hyb[h] = spp.compare(spp.oracle_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3, hybrid=h), orc)
        print(f"hybrid {h}: {time.time() - t0:.1f} s {hyb[h]['same_run']}", file=sys.stderr, flush=True)
    if a.hybrid_only:
        print(json.dumps({"case": a.case, "n": a.n, "engine": {k: eng[k] for k in KEYS},
                          "hybrid_solves": {k: hyb[1][k] for k in KEYS},
                          "hybrid_solves_fused": {k: hyb[2][k] for k in KEYS}}, indent=1))
        return
    draws = []
    for d in range(spp.FLOOR_DRAWS):
        draws.append(spp.compare(spp.floor_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3, d), orc))
        print(f"floor draw {d}: {time.time() - t0:.1f} s {draws[-1]['same_run']}", file=sys.stderr,
              flush=True)
    out = {"case": a.case, "n": a.n, "engine": {k: eng[k] for k in KEYS},
           "hybrid_solves": {k: hyb[1][k] for k in KEYS},
           "hybrid_solves_fused": {k: hyb[2][k] for k in KEYS},
           "draws": [{k: d[k] for k in KEYS} for d in draws], "summary": {}}
    for k in KEYS:
        v = [d[k] for d in draws]
        mu = sum(v) / len(v)
        sd = math.sqrt(sum((x - mu) ** 2 for x in v) / (len(v) - 1))
        se = math.sqrt(max(mu * (1 - mu), 1e-12) / a.n)
        out["summary"][k] = {"engine": eng[k], "draws_min": min(v), "draws_mean": mu, "draws_sd": sd,
                             "binomial_se": se, "engine_minus_mean_in_sd": (eng[k] - mu) / max(sd, 1e-12),
                             "engine_minus_min": eng[k] - min(v), "bound": spp.floor_bound(draws, k, a.n)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
