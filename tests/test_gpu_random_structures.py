"""The HIP engine on sparse QPs that are not the MPC problem: random banded P, random A patterns,
feasible boxes with equality rows, a batch of value sets per pattern, both solve-step kinds (paired:
segments 0 + 1 of a lane share one LDS atomic; unpaired: four atomics; MPCQP_PAIRED forces the
planner).  Parity with the oracle (OSQP 0.6 restated, oracle/osqp_oracle.c) at eps 1e-5: statuses
and iteration counts identical (measured on MI355X: 4 x 96 of 4 x 96), solutions within 1e-6."""
import numpy as np
import pytest
import scipy.sparse as sp

import oracle as orc
from mpc_arpo_project_amd.engine import BatchQP

pytestmark = pytest.mark.gpu


def _random_qp(seed, B):
    rng = np.random.default_rng(500 + seed)
    n, m = 70 + 13 * seed, 110 + 17 * seed
    off = rng.uniform(-0.3, 0.3, n - 1)
    P = sp.diags([off, 2.0 + rng.random(n), off], [-1, 0, 1], format="csc")
    rows, cols = [], []
    for i in range(m):
        for j in rng.choice(n, size=int(rng.integers(2, 6)), replace=False):
            rows.append(i), cols.append(int(j))
    A = sp.csc_matrix((np.ones(len(rows)), (rows, cols)), shape=(m, n))
    A.sum_duplicates()
    A.sort_indices()
    q = rng.standard_normal(n)
    Ax = rng.standard_normal((B, A.nnz))
    l, u = np.empty((B, m)), np.empty((B, m))
    for b in range(B):
        Ab = sp.csc_matrix((Ax[b], A.indices, A.indptr), shape=A.shape)
        x0 = rng.standard_normal(n)
        c = Ab @ x0
        w = rng.uniform(0.1, 1.0, m)
        eq = rng.random(m) < 0.2
        w[eq] = 0.0
        l[b], u[b] = c - w, c + w
    return P, q, A, Ax, l, u


@pytest.mark.parametrize("waves", ["0", "2", "3"])
@pytest.mark.parametrize("paired", ["1", "0"])
@pytest.mark.parametrize("seed", [1, 2])
def test_random_structures_match_oracle(monkeypatch, paired, seed, waves):
    """waves: MPCQP_WAVES -- 0 the automatic choice (one wave for these sizes), 2 two waves with the
    solve steps split between them (their own step packing), 3 two waves with the steps on the first
    (Two waves per instance)"""
    monkeypatch.setenv("MPCQP_DIAGNOSTICS", "1")  # the overrides are diagnostics
    monkeypatch.setenv("MPCQP_PAIRED", paired)
    monkeypatch.setenv("MPCQP_WAVES", waves)
    B = 96
    P, q, A, Ax, l, u = _random_qp(seed, B)
    st = dict(eps_abs=1e-5, eps_rel=1e-5)
    qp = BatchQP(P, A, batch=B, **st)
    qp.set_data(q=q, Ax=Ax, l=l, u=u)
    r = qp.solve()
    xo, yo, so, io = orc.batch_solve(P, q, A, Ax, l, u, nthreads=8, **st)
    sg, ig, xg = r.status.cpu().numpy(), r.iter.cpu().numpy(), r.x.cpu().numpy()
    print(f"waves={waves} paired={paired} seed={seed}: statuses {np.unique(so, return_counts=True)}, "
          f"status agreement {np.mean(sg == so):.4f}, iteration agreement {np.mean(ig == io):.4f}")
    assert np.mean(so == 1) >= 0.9  # the generator makes feasible, well-posed QPs
    assert np.array_equal(sg, so)
    assert np.array_equal(ig, io)
    ok = (so == 1) & (sg == 1)
    assert np.max(np.abs(xg[ok] - xo[ok]) / (1 + np.abs(xo[ok]))) < 1e-6
