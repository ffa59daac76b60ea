"""The CPU oracle (oracle/osqp_oracle.c, restatement of OSQP 0.6) against fixtures and KKT
certificates.  OSQP itself is unavailable, so the oracle is pinned by (1) the reference's own
QP data, (2) independently KKT-certified polished solutions, (3) an LP feasibility check of the
instances it declares primal infeasible (scipy linprog)."""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp
from scipy.optimize import linprog

import oracle as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def _setup(d):
    P = sp.csc_matrix((d["P_data"], d["P_indices"], d["P_indptr"]), shape=tuple(d["P_shape"]))
    A = sp.csc_matrix((d["A_data"], d["A_indices"], d["A_indptr"]), shape=tuple(d["A_shape"]))
    return P, d["q"], A


def test_oracle_regression_first_solve(golden):
    d = golden("cl_n20")
    P, q, A = _setup(d)
    s = orc.OracleOSQP()
    s.setup(P, q, A, d["l"], d["u"], warm_start=True, verbose=False)
    r = s.solve()
    assert r.info.status == "solved"
    assert r.info.iter == d["solve_iter"][0]
    assert np.array_equal(r.x, d["solve_x"][0])


def _cert_inputs(tag):
    import gen_certs as gc

    c = np.load(os.path.join(GOLDEN, f"cert256_{tag}.npz"), allow_pickle=False)
    prob, X, Ax, l, u = gc.inputs(tag)
    assert gc.digest(Ax, l, u) == str(c["sha256"]), "regenerated QPs differ from the certified ones"
    return gc, c, prob, Ax, l, u


@pytest.mark.parametrize("tag", ["n20", "n40dv"])
def test_certificates_hold(tag):
    """the committed optima of >= 248 instances per config satisfy the KKT conditions of the
    regenerated QPs to 1e-9 (primal feasibility, stationarity, complementarity)"""
    gc, c, prob, Ax, l, u = _cert_inputs(tag)
    assert len(c["idx"]) >= 248
    P = sp.csc_matrix(prob.P)
    Pfull = P + sp.triu(P, 1).T if sp.tril(P, -1).nnz == 0 else P
    for k, b in enumerate(c["idx"]):
        A = sp.csc_matrix((Ax[b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
        cert = gc.certify(Pfull, prob.q, A, l[b], u[b], c["x"][k], c["y"][k])
        assert max(cert) <= 1e-9, (b, cert)


@pytest.mark.parametrize("tag", ["n20", "n40dv"])
def test_oracle_admm_converges_to_certified_optimum(tag):
    """the oracle's ADMM (no polish) converges to the independently certified optimum as eps
    shrinks: at eps = 1e-9 every certified instance is solved with |u0 - u0*| < 1e-6 (measured
    max 2.2e-7 / 9.8e-8), and the median error falls by >= 1e3 from eps 1e-4 to 1e-9"""
    gc, c, prob, Ax, l, u = _cert_inputs(tag)
    idx = c["idx"]
    med = {}
    for eps, mi in ((1e-4, 4000), (1e-9, 400000)):
        x, _, st, _ = orc.batch_solve(prob.P, prob.q, prob.A, Ax[idx], l[idx], u[idx], nthreads=8,
                                      eps_abs=eps, eps_rel=eps, max_iter=mi)
        du = np.abs(x[:, prob.u0_slice] - c["u0"]).max(axis=1)
        if eps == 1e-9:
            assert np.all(st == 1)
            assert du.max() < 1e-6, du.max()
        med[eps] = float(np.median(du[st == 1]))
    assert med[1e-9] * 1e3 < med[1e-4], med


def test_oracle_primal_infeasible_is_infeasible(golden, prob20):
    d = golden("batch_n20")
    P, q = prob20.P, prob20.q
    x, y, st, it = orc.batch_solve(P, q, prob20.A, d["Ax"][:16], d["l"][:16], d["u"][:16],
                                   nthreads=4, eps_abs=1e-4, eps_rel=1e-4)
    n = prob20.n
    for b in np.nonzero(st == -3)[0][:3]:
        A = sp.csc_matrix((d["Ax"][b], d["A_indices"], d["A_indptr"]), shape=prob20.A.shape)
        lo, hi = d["l"][b], d["u"][b]
        fin_u, fin_l = np.isfinite(hi), np.isfinite(lo)
        A_ub = sp.vstack([A[fin_u], -A[fin_l]]).tocsr()
        b_ub = np.hstack([hi[fin_u], -lo[fin_l]])
        res = linprog(np.zeros(n), A_ub=A_ub, b_ub=b_ub, bounds=[(None, None)] * n, method="highs")
        assert res.status == 2, "oracle says infeasible, LP says feasible"
    for b in np.nonzero(st == 1)[0][:3]:
        assert np.all(np.isfinite(x[b]))


def test_oracle_settings_semantics(golden, prob20):
    d = golden("batch_n20")
    b = 0
    A = sp.csc_matrix((d["Ax"][b], d["A_indices"], d["A_indptr"]), shape=prob20.A.shape)
    s = orc.OracleOSQP()
    s.setup(prob20.P, prob20.q, A, d["l"][b], d["u"][b], max_iter=30, eps_abs=1e-9, eps_rel=1e-9)
    r = s.solve()
    assert r.info.status in ("maximum iterations reached", "solved inaccurate")
    assert r.info.iter == 30
    with pytest.raises(ValueError):
        s.update(l=d["u"][b] + 1.0, u=d["u"][b])
