"""Modelled step count of two-atomic ("quad") solve steps on the chosen plan's solve levels (host
only).  A quad lane sums segments 0+1 and 2+3 into two targets, so a step holds at most 128
target units of <= 2 segments; the paired step holds 256 segments (64 pairs + 128 singles).
usage: python tools/quad_count.py 20 0   (Nx, delta-v)"""
import math
import os
import subprocess
import sys

if os.environ.get("QC_CHILD"):
    import numpy as np

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
    from conftest import problem
    from mpc_arpo_project_amd import _lib
    from mpc_arpo_project_amd.engine import sorted_csc, triu_csc

    prob = problem(int(sys.argv[1]), sys.argv[2] == "1")
    P, A = triu_csc(prob.P), sorted_csc(prob.A)
    _lib.schedule_check(P, A, 1e-6, np.ones(A.shape[0]), np.ones(P.shape[0] + A.shape[0]))
    sys.exit(0)

env = dict(os.environ, QC_CHILD="1", MPCQP_DUMP_CAPS="1", MPCQP_DUMP_TASKS="1", MPCQP_NO_ANNEAL="1")
err = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=env, capture_output=True,
                     text=True, check=True).stderr.splitlines()
i = max(k for k, l in enumerate(err) if l.startswith("caps"))  # the final build's levels follow
print(err[i])
tp = tq = 0
for l in err[i + 1:]:
    if not l.startswith("level:"):
        continue
    segs = [math.ceil(int(t[1:]) / 2) for t in l.split()[1:]]
    S, units = sum(segs), sum(math.ceil(s / 2) for s in segs)
    p, q = max(math.ceil(S / 256), 1), math.ceil(units / 128)
    tp, tq = tp + p, tq + q
    print(f"tasks {len(segs):4d} segments {S:4d} quad units {units:4d}: paired >= {p}, quad {q}")
print(f"steps per ADMM iteration: paired >= {tp}, quad {tq}")
