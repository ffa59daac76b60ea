"""Records the warm closed loop of tests/test_gpu_scale_parity.py::lockstep (GPU): per step the QP
data (Ax, l, u), the engine's warm state before the solve and its status / iterations after it, so
that tools/lockstep_floor.py can measure on the CPU how much the oracle itself moves under a 1-ulp
perturbation of that state.   python tools/lockstep_record.py B K out.npz
"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import problem
from mpc_arpo_project_amd import scenarios
from mpc_arpo_project_amd.closed_loop import BatchClosedLoop

B, K, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
prob = problem(20, False)
X = scenarios.sample_estimates(2048, seed=20250328)[:B, :4].copy(); X[:, 2:4] = 0.0
cl = BatchClosedLoop(prob, X, eps_abs=1e-4, eps_rel=1e-4)
rec = {k: [] for k in ("Ax", "l", "u", "x", "z", "y", "rho", "hs", "st", "it")}
for k in range(K):
    Ax, l, u = (t.cpu().numpy() for t in cl.qp.copy_data())
    s = {key: v.cpu().numpy() for key, v in cl.qp.get_state().items()}
    r = cl.step()
    for key, val in (("Ax", Ax), ("l", l), ("u", u), ("x", s["x"]), ("z", s["z"]), ("y", s["y"]),
                     ("rho", s["rho"]), ("hs", s["has_state"]), ("st", r.status.cpu().numpy()),
                     ("it", r.iter.cpu().numpy())):
        rec[key].append(np.array(val))
cl.close()
np.savez_compressed(out, **{k: np.stack(v) for k, v in rec.items()})
print("recorded", B, K)
