"""The CPU oracle (oracle/osqp_oracle.c, restatement of OSQP 0.6) against fixtures and KKT
certificates.  OSQP itself is unavailable, so the oracle is pinned by (1) the reference's own
QP data, (2) independently KKT-certified polished solutions, (3) an LP feasibility check of the
instances it declares primal infeasible (scipy linprog)."""
import numpy as np
import pytest
import scipy.sparse as sp
from scipy.optimize import linprog

import oracle as orc


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


def test_oracle_certified_solutions(golden, prob20):
    """polished solutions satisfy KKT to 1e-8; an eps=1e-6 ADMM solve lands within 1e-5 in u0"""
    d = golden("batch_n20")
    c = golden("cert_batch_n20")
    P, q = prob20.P, prob20.q
    sl = prob20.u0_slice
    checked = 0
    for b in range(8):
        if not np.all(np.isfinite(c["x"][b])) or np.max(c["cert"][b]) > 1e-8:
            continue
        A = sp.csc_matrix((d["Ax"][b], d["A_indices"], d["A_indptr"]), shape=prob20.A.shape)
        s = orc.OracleOSQP()
        s.setup(P, q, A, d["l"][b], d["u"][b], eps_abs=1e-6, eps_rel=1e-6, max_iter=20000)
        r = s.solve()
        assert np.max(np.abs(r.x[sl] - c["x"][b][sl])) < 1e-5
        checked += 1
    assert checked >= 3


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
