"""Engine-driven vs oracle-driven full-length sweeps (tests/sweep_parity.py), with the oracle's
own one-ulp floor, for the sweep configurations of DESIGN.md (Parity): prints one JSON object.

    python tools/sweep_parity.py [--n 256] > profiles/<round>/sweep_parity.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import sweep_parity as spp  # noqa: E402
from mpc_arpo_project_amd import sweep  # noqa: E402

CASES = {
    # the sweep driver's defaults: radial, N = 20, noise 0.3 held 50 samples, rejection on
    "radial_n20_noise": dict(scenario="radial", Nx=20, noise=(0.3, 0.3, 50), isReject=True,
                             T_final=150.0),
    # test/traj_eval_in_track.py: in-track, N = 40, no noise, no rejection
    "in_track_n40": dict(scenario="in_track", Nx=40, noise=None, isReject=False, T_final=150.0),
}


def run_case(name, n, eps=1e-3):
    c = CASES[name]
    sim, prob = sweep.build(c["scenario"], c["Nx"], c["noise"], c["isReject"], c["T_final"])
    nsim = int(sim.T_final / sim.time_stp)
    X0 = sweep.initial_conditions(c["scenario"], n)
    t0 = time.time()
    e = spp.engine_run(prob, X0, nsim, sim.suc_cond, c["noise"], eps)
    t1 = time.time()
    o = spp.oracle_run(prob, X0, nsim, sim.suc_cond, c["noise"], eps)
    t2 = time.time()
    o1 = spp.floor_run(prob, X0, nsim, sim.suc_cond, c["noise"], eps, 0)
    return dict(case=name, config=dict(c, eps=eps, nsim=nsim), n=n,
                engine_vs_oracle=spp.compare(e, o), oracle_vs_oracle_ulp=spp.compare(o1, o),
                seconds=dict(engine=t1 - t0, oracle=t2 - t1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--cases", default=",".join(CASES))
    a = ap.parse_args()
    out = [run_case(k, a.n) for k in a.cases.split(",")]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
