"""Which plan choice moves the engine's closed loops away from the oracle's?
One full-length sweep case, the oracle-driven run and two of its one-ulp floor draws computed once,
then the engine-driven run under several planner settings (environment switches read at create
time: MPCQP_COPY_ROWS -- 0 round-2 copies, 1 exact copy rows only, 4 default with the last-level
fold; MPCQP_CAPM / MPCQP_CAPW -- block caps of the blocked substitution).  Prints one JSON object.

    python tools/plan_parity.py [--case radial20] [--n 1024] > profiles/r04/plan_parity.json
"""
import argparse
import json
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
}
VARIANTS = [
    ("default", {}),
    ("copy_rows_only", {"MPCQP_COPY_ROWS": "1"}),
    ("round2_copies", {"MPCQP_COPY_ROWS": "0"}),
    ("caps_96_320", {"MPCQP_CAPM": "96", "MPCQP_CAPW": "320"}),
    ("caps_128_384", {"MPCQP_CAPM": "128", "MPCQP_CAPW": "384"}),
]
KEYS = ("same_run", "i_term_agree", "success_agree")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="radial20", choices=sorted(CASES))
    ap.add_argument("--n", type=int, default=1024)
    a = ap.parse_args()
    scen, nx, noise, rej, tf = CASES[a.case]
    sim, prob = sweep.build(scen, nx, noise, rej, tf)
    nsim = int(sim.T_final / sim.time_stp)
    X0 = sweep.initial_conditions(scen, a.n)
    t0 = time.time()
    orc = spp.oracle_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3)
    print(f"oracle run: {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    floors = {}
    for d in (0, 2):
        floors[f"draw{d}"] = spp.compare(spp.floor_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3, d), orc)
        print(f"floor draw {d}: {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    out = {"case": a.case, "n": a.n, "floor": {k: {q: v[q] for q in KEYS} for k, v in floors.items()},
           "engine": {}}
    for name, env in VARIANTS:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            from mpc_arpo_project_amd.closed_loop import BatchClosedLoop
            probe = BatchClosedLoop(prob, X0[:8])
            sched = probe.qp.schedule_info()
            probe.close()
            e = spp.engine_run(prob, X0, nsim, sim.suc_cond, noise, 1e-3)
            c = spp.compare(e, orc)
            out["engine"][name] = dict(env=env, steps=sched["fwd_steps"] + sched["bwd_steps"],
                                       lds_bytes=sched["lds_bytes"], **{q: c[q] for q in KEYS})
            print(name, out["engine"][name], file=sys.stderr, flush=True)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
