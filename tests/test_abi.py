"""libmpcqp.so loads and exports every symbol include/*.h declares; host-only entry points work
without a GPU (no compute call is made here)."""
import ctypes as C
import glob
import os
import re

import numpy as np

from mpc_arpo_project_amd import _lib
from mpc_arpo_project_amd.engine import triu_csc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        names |= set(re.findall(r"^(?:int|const char \*)\s*(mpcqp_\w+)\(", src, re.M))
    return names


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    declared = _declared()
    assert len(declared) >= 20
    missing = [n for n in declared if not hasattr(L, n)]
    assert not missing, missing
    assert declared == set(_lib.EXPORTED)


def test_host_only_entry_points():
    L = _lib.lib()
    assert L.mpcqp_version() >= 100
    s = _lib.default_settings()
    assert (s.rho, s.sigma, s.alpha, s.max_iter, s.check_termination) == (0.1, 1e-6, 1.6, 4000, 25)
    assert L.mpcqp_status_string(1) == b"solved"
    assert L.mpcqp_status_string(-2) == b"maximum iterations reached"
    assert L.mpcqp_status_string(-3) == b"primal infeasible"


def test_symbolic_analysis_matches_oracle_factor(prob20):
    """the engine's KKT ordering/factor pattern equals the oracle's QDLDL factor size"""
    import oracle as orc

    perm, Lp, Li, st = _lib.analyze(triu_csc(prob20.P), prob20.A)
    s = orc.OracleOSQP()
    s.setup(prob20.P, prob20.q, prob20.A, prob20.l, prob20.u)
    assert len(Li) == s.state()["nnzL"] == 1313
    assert sorted(perm.tolist()) == list(range(prob20.n + prob20.m))
    # L strictly lower, sorted columns
    for j in range(len(Lp) - 1):
        col = Li[Lp[j]:Lp[j + 1]]
        assert np.all(col > j) and np.all(np.diff(col) > 0)
    # blocked substitution: a handful of blocks instead of the 81-level elimination chain; with the
    # balanced accumulation placement and the per-structure block caps, 13 serial 64-lane steps per
    # ADMM iteration, inside the 40 KB that keeps 4 instances per CU
    assert st["fwd_levels"] <= 8 and st["fwd_steps"] + st["bwd_steps"] <= 13
    assert st["lds_image_bytes"] <= 160 * 1024 // 4


def test_invalid_structure_rejected():
    P = np.array([[1.0, 0.0], [1.0, 1.0]])
    import scipy.sparse as sp

    Pl = sp.csc_matrix(np.tril(P))  # lower triangle: must be refused
    A = sp.csc_matrix(np.eye(2))
    try:
        _lib.analyze(Pl, A)
    except _lib.MPCQPError as e:
        assert "upper" in str(e)
    else:
        raise AssertionError("lower-triangular P accepted")


def test_horizon_limits():
    """the reference's horizons (Nx 20-50) are planned; structures beyond the (4, 8)
    register bucket (Nx > 51 for the planar model) are refused at analysis / create time instead
    of running a spill-bound instantiation"""
    from conftest import problem

    for nx in (50, 51):
        p = problem(nx, False)
        _, _, _, st = _lib.analyze(triu_csc(p.P), p.A)
        assert st["fwd_steps"] > 0
    p = problem(52, False)
    try:
        _lib.analyze(triu_csc(p.P), p.A)
    except _lib.MPCQPError as e:
        assert "too large" in str(e)
    else:
        raise AssertionError("Nx = 52 accepted")


def test_plan_overrides_need_the_diagnostics_switch(prob20, monkeypatch):
    """the MPCQP_* plan / kernel overrides are diagnostics: without MPCQP_DIAGNOSTICS=1 an inherited
    override (here block caps that change the plan) is ignored and the validated plan is built"""
    _, _, _, st0 = _lib.analyze(triu_csc(prob20.P), prob20.A)
    monkeypatch.setenv("MPCQP_CAPM", "96")
    monkeypatch.setenv("MPCQP_CAPW", "320")
    monkeypatch.delenv("MPCQP_DIAGNOSTICS", raising=False)
    _, _, _, st1 = _lib.analyze(triu_csc(prob20.P), prob20.A)
    assert st1 == st0
    monkeypatch.setenv("MPCQP_DIAGNOSTICS", "1")
    _, _, _, st2 = _lib.analyze(triu_csc(prob20.P), prob20.A)
    assert st2 != st0  # the override is honoured with the switch (caps 96/320, 16 steps)
