"""CPU side of tools/lockstep_record.py: per step of the recorded warm closed loop, the oracle's
warm solve from the engine's state (as in the lockstep test) and from that state moved by one ulp;
prints the engine-vs-oracle and the oracle-vs-oracle(1 ulp) status agreement per step.
    python tools/lockstep_floor.py rec.npz [threads]
"""
import os, sys
import numpy as np
import scipy.sparse as sp
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle")); sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle as orc
from conftest import problem

d = np.load(sys.argv[1]); th = int(sys.argv[2]) if len(sys.argv) > 2 else 8
prob = problem(20, False)
K, B = d["st"].shape
rng = np.random.default_rng(7)
def ulp(a):
    up = rng.random(a.shape) < 0.5
    return np.where(up, np.nextafter(a, np.inf), np.nextafter(a, -np.inf))
def make(k):
    ss = []
    for b in range(B):
        A = sp.csc_matrix((d["Ax"][k][b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
        s = orc.OracleOSQP(); s.setup(prob.P, prob.q, A, d["l"][k][b], d["u"][k][b], eps_abs=1e-4,
                                      eps_rel=1e-4, warm_start=True, verbose=False)
        ss.append(s)
    return ss
ge, oo = [], []
s1, s2 = make(0), make(0)
for ss in (s1, s2):
    orc.batch_update_solve(ss, None, None, None, th)
for k in range(1, K):
    orc.batch_set_state(s1, d["x"][k], d["z"][k], d["y"][k], d["rho"][k])
    orc.batch_set_state(s2, ulp(d["x"][k]), ulp(d["z"][k]), ulp(d["y"][k]), d["rho"][k])
    _, so1, io1 = orc.batch_update_solve(s1, d["Ax"][k], d["l"][k], d["u"][k], th)
    _, so2, io2 = orc.batch_update_solve(s2, d["Ax"][k], d["l"][k], d["u"][k], th)
    ge.append(float(np.mean(so1 == d["st"][k]))); oo.append(float(np.mean(so1 == so2)))
    print(k, "engine vs oracle", round(ge[-1], 4), " oracle vs oracle(1ulp)", round(oo[-1], 4), flush=True)
print("mean engine-vs-oracle", np.mean(ge), "mean oracle-vs-oracle(1ulp)", np.mean(oo))
