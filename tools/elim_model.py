"""Planner model of eliminating the always-free rows (l = -inf, u = +inf: the -inf x (Nx - Nb) ny
block of reference src/simhelpers.py:137-138) from the KKT system (VERDICT r02 item
2): the reduced system [[P + sigma I + sum_free rho_i a_i' a_i, A_k'], [A_k, -diag(1/rho_k)]]
(the free rows folded in exactly through their Schur complement) has the pattern of
P + A_free' A_free next to the kept rows.  Prints nnz(L), triangular-solve steps, factorization
steps and the LDS image of the engine's planner for the full and the reduced structure.

    python tools/elim_model.py > profiles/r03/elim_model.json
"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import problem  # noqa: E402
from mpc_arpo_project_amd import _lib  # noqa: E402
from mpc_arpo_project_amd.engine import sorted_csc, triu_csc  # noqa: E402


def plan(P, A):
    perm, Lp, Li, st = _lib.analyze(triu_csc(P), sorted_csc(A))
    return dict(n=P.shape[0], m=A.shape[0], kkt=P.shape[0] + A.shape[0], nnzL=int(Lp[-1]), **st)


out = {}
for Nx, dv in [(20, False), (40, True)]:
    prob = problem(Nx, dv)
    A = sp.csc_matrix(prob.A)
    free = (prob.l < -1e20) & (prob.u > 1e20)
    Af = A[free]
    Pn = sp.csc_matrix(prob.P) + Af.T @ Af  # pattern of P + A_free' A_free
    Pn = sp.csc_matrix((np.ones(Pn.nnz), Pn.indices, Pn.indptr), shape=Pn.shape)
    out[f"N{Nx}{'_dv' if dv else ''}"] = dict(free_rows=int(free.sum()), full=plan(prob.P, A),
                                             reduced=plan(Pn, A[~free]))
print(json.dumps(out, indent=1))
