"""Per-(step, chaser) ADMM iterations of the default bench workload (B = 65,536, N = 20: the cold
step, 4 warm steps, 20 timed steps), saved for the offline schedule simulation
(tools/sched_sim.py).  usage (GPU box): python tools/iters_dump.py out.npz"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from mpc_arpo_project_amd import qp_model, scenarios  # noqa: E402
from mpc_arpo_project_amd.closed_loop import BatchClosedLoop  # noqa: E402

nx = int(os.environ.get("NX", 20))
dv = os.environ.get("DV", "0") == "1"
sim, mpc, fail, deb = scenarios.radial_scenario(Nx=nx, isDeltaV=dv)
prob = qp_model.build_problem(sim, mpc, fail, deb)
B = 65536
X0 = bench.initial_states(B, 0, B, 20250328)
cl = BatchClosedLoop(prob, X0, device="cuda", eps_abs=1e-4, eps_rel=1e-4)
its, act = [], []
for k in range(25):
    a = (cl.done == 0).cpu().numpy()
    r = cl.step()
    its.append(r.iter.cpu().numpy().astype(np.int16))
    act.append(a)
    print(k, float(r.iter.float()[torch.as_tensor(a, device='cuda')].mean()), flush=True)
np.savez_compressed(sys.argv[1], iters=np.array(its), active=np.array(act))
