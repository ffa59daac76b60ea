"""The compiled device program, checked on the CPU (no GPU): mpcqp_schedule_check interprets the
exact schedules mpcqp_create uploads -- KKT assembly, factorization with its group butterflies,
the block-inverse tail, one forward / diagonal / backward solve -- and the result must solve the
KKT system [[P + sigma I, A'], [A, -diag(1/rho)]] (OSQP 0.6 kkt.c form_KKT, the system the
reference's osqp solves every ADMM iteration).  This pins the symbolic compiler and the LDS layout
optimiser (csrc/lds_layout.cpp): every slot relabelling, segment move, operand flip and sink they
make must leave the solve exact to rounding.  The LDS cost model is checked to be below the
unoptimised layout's."""
import numpy as np
import pytest
import scipy.sparse as sp

from mpc_arpo_project_amd import _lib
from mpc_arpo_project_amd.engine import sorted_csc, triu_csc


def _kkt(P, A, sigma, rho):
    n, m = P.shape[0], A.shape[0]
    Pf = sp.csc_matrix(P)
    return sp.bmat([[Pf + sigma * sp.eye(n), A.T], [A, -sp.diags(1.0 / rho)]], format="csc")


@pytest.mark.parametrize("waves", ["1", "2", "3"])
@pytest.mark.parametrize("Nx,dv", [(20, False), (40, True), (30, False), (40, False), (50, True),
                                   (51, False)])
def test_emulated_schedule_solves_kkt(monkeypatch, Nx, dv, waves):
    """waves 2: the plan laid out for two waves per instance (every target of a step in one half
    of the segment positions, symbolic.cpp) solves the same system; the other horizons of the
    reference's scripts (Nx 20-50) up to the largest the (4, 8) bucket accepts"""
    from conftest import problem

    monkeypatch.setenv("MPCQP_DIAGNOSTICS", "1")  # the overrides are diagnostics
    monkeypatch.setenv("MPCQP_WAVES", waves)

    prob = problem(Nx, dv)
    P, A = triu_csc(prob.P), sorted_csc(prob.A)
    rng = np.random.default_rng(Nx)
    for trial in range(3):
        # the bench's P, random A values on A's pattern, rho over the adaptive-rho range with
        # OSQP's equality class (1e3 rho)
        Ax = A.copy()
        Ax.data = prob.A.tocsc().sorted_indices().data * (1 + 0.1 * rng.standard_normal(A.nnz))
        rho = 10.0 ** rng.uniform(-3, 2, A.shape[0])
        rho[: A.shape[0] // 4] *= 1e3
        sigma = 1e-6
        rhs = rng.standard_normal(P.shape[0] + A.shape[0])
        sol, model = _lib.schedule_check(P, Ax, sigma, rho, rhs)
        K = _kkt(P + sp.triu(P, 1).T, Ax, sigma, rho)
        ref = sp.linalg.spsolve(K, rhs)
        rel = np.abs(sol - ref).max() / np.abs(ref).max()
        res = np.abs(K @ sol - rhs).max() / np.abs(rhs).max()
        assert rel < 1e-8 and res < 1e-9, (trial, rel, res)


def test_layout_optimiser_lowers_modelled_lds_cycles(monkeypatch):
    """the annealed layout (default) models fewer LDS cycles than the greedy one it starts from"""
    from conftest import problem

    prob = problem(20, False)
    P, A = triu_csc(prob.P), sorted_csc(prob.A)
    args = (P, A, 1e-6, np.ones(A.shape[0]), np.ones(P.shape[0] + A.shape[0]))
    _, opt = _lib.schedule_check(*args)
    monkeypatch.setenv("MPCQP_DIAGNOSTICS", "1")  # the overrides are diagnostics
    monkeypatch.setenv("MPCQP_NO_ANNEAL", "1")
    _, greedy = _lib.schedule_check(*args)
    tot = lambda d: d["read"] + d["atomic"] + d["vec"]
    # 12 solve steps (6 + 6: identity terms folded into W's start values) of 32 reads + 12 atomic
    # cycles, 6 register slots of vector passes
    assert opt["floor"] == greedy["floor"] == 12 * 44 + 6 * 10
    assert tot(opt) < 0.8 * tot(greedy), (opt, greedy)


@pytest.mark.parametrize("waves", ["1", "2", "3"])
@pytest.mark.parametrize("copy_rows", ["4", "2", "0"])
@pytest.mark.parametrize("paired", ["0", "1"])
@pytest.mark.parametrize("seed", [1, 2])
def test_emulated_schedule_random_structures(monkeypatch, paired, seed, copy_rows, waves):
    """both step kinds (paired: segments 0 + 1 of a lane on one target, 3 atomics; unpaired: 4)
    solve the KKT system of random sparse QPs, not only the MPC structure the planner was tuned on;
    with the product's copy rows and last-level fold (4), the identity term folded everywhere (2)
    and block-0 copy rows only (0)"""
    monkeypatch.setenv("MPCQP_DIAGNOSTICS", "1")  # the overrides are diagnostics
    monkeypatch.setenv("MPCQP_PAIRED", paired)
    monkeypatch.setenv("MPCQP_COPY_ROWS", copy_rows)
    monkeypatch.setenv("MPCQP_WAVES", waves)
    rng = np.random.default_rng(100 + seed)
    n, m = 70 + 13 * seed, 110 + 17 * seed
    # within the residual layout's widths (rows of A <= 8 terms, symmetric rows of P <= 4)
    off = rng.uniform(-0.3, 0.3, n - 1)
    P = sp.diags([off, 2.0 + rng.random(n), off], [-1, 0, 1], format="csc")
    rows, cols = [], []
    for i in range(m):
        for j in rng.choice(n, size=int(rng.integers(2, 6)), replace=False):
            rows.append(i), cols.append(int(j))
    A = sp.csc_matrix((rng.standard_normal(len(rows)), (rows, cols)), shape=(m, n))
    P, A = triu_csc(P), sorted_csc(A)
    rho = 10.0 ** rng.uniform(-2, 2, m)
    sigma = 1e-6
    rhs = rng.standard_normal(n + m)
    sol, model = _lib.schedule_check(P, A, sigma, rho, rhs)
    K = _kkt(P + sp.triu(P, 1).T, A, sigma, rho)
    ref = sp.linalg.spsolve(K, rhs)
    rel = np.abs(sol - ref).max() / np.abs(ref).max()
    res = np.abs(K @ sol - rhs).max() / np.abs(rhs).max()
    assert rel < 1e-8 and res < 1e-9, (rel, res)
    assert model["floor"] > 0
