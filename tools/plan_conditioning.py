"""Backward error of the engine's KKT solves per plan, on the CPU.

The engine's triangular solves are a blocked substitution, w_R = M_R c_R - G_R w_{R-1} with
M_R = L_RR^-1 precomputed (Schedules): multiplying by an explicit block inverse is not
backward stable the way QDLDL's row-by-row substitution is, and its error depends on the block
partition the planner picks.  This tool measures it on the KKT systems the closed loop really
factorizes:

  * instances: the reference's recorded closed-loop update sequences (tests/golden/cl_n20,
    cl_noise_n20, cl_n40dv: every warm step) replayed through the oracle (OSQP 0.6 restated, CPU);
    after each solve the oracle's scaling (D, E, c), rho and scaled iterates give the scaled KKT
    matrix K = [[c D P D + sigma I, (E A D)'], [E A D, -diag(1 / rho_vec)]] and the right-hand
    side of the next ADMM iteration [sigma x - c D q; z - y / rho_vec];
  * omega = max_i |K x - b|_i / (|K| |x| + |b|)_i, the componentwise backward error (a backward
    stable substitution keeps it at a few ulps);
  * for each plan (block caps, step kind; MPCQP_* diagnostics), the compiled device program run
    by the CPU interpreter (mpcqp_schedule_check on the host-only library, tools/sanitize/Makefile
    `host`) solves every instance; omega against the same number for an unblocked plan (every block one row:
    plain level-scheduled substitution, QDLDL's arithmetic up to summation order) and for SuperLU;
  * per plan the growth of its block inverses, max_R ||M_R||_inf ||L_RR||_inf, is not exported by
    the planner; the backward error is the quantity that matters for the closed loops.

usage: python tools/plan_conditioning.py [--out profiles/r05/plan_conditioning.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

HOST_LIB = os.path.join(REPO, "build", "host", "libmpcqp_host.so")

RHO_MIN, RHO_EQ, RHO_TOL, INF = 1e-6, 1e3, 1e-4, 1e30
SIGMA = 1e-6


def rho_vec(rho, l, u):
    """auxil.c set_rho_vec on scaled bounds"""
    r = np.full(l.shape, rho)
    free = (l < -INF * 1e-4) & (u > INF * 1e-4)
    eq = ~free & (u - l < RHO_TOL)
    r[eq] = RHO_EQ * rho
    r[free] = RHO_MIN
    return r


def instances(tag, limit=None):
    """warm KKT systems of the reference's recorded closed loop `tag` (module docstring)"""
    import oracle as orc
    from conftest import load_golden

    d = load_golden(tag)
    if "P_data" in d:
        P = sp.csc_matrix((d["P_data"], d["P_indices"], d["P_indptr"]), shape=tuple(d["P_shape"]))
        A = sp.csc_matrix((d["A_data"], d["A_indices"], d["A_indptr"]), shape=tuple(d["A_shape"]))
        q, l0, u0 = d["q"], d["l"], d["u"]
    else:  # cl_noise_n20: the N = 20 problem with this run's set-up bounds
        from conftest import problem
        pr = problem(20, False)
        P = sp.csc_matrix(pr.P)
        A = sp.csc_matrix((d["A_data"], pr.A.indices, pr.A.indptr), shape=pr.A.shape)
        q, l0, u0 = pr.q, d["setup_l"], d["setup_u"]
    P = sp.triu(P, format="csc")
    P.sort_indices()
    A.sort_indices()
    s = orc.OracleOSQP()
    s.setup(P, q, A, l0, u0, warm_start=True, verbose=False)
    out = []
    steps = d["step_Ax"].shape[0]
    for i in range(steps if limit is None else min(limit, steps)):
        s.solve()
        st = s.state()
        D, E, c, rho = st["D"], st["E"], st["c"], st["rho"]
        Ai = sp.csc_matrix((d["step_Ax"][i - 1] if i else A.data, A.indices, A.indptr), shape=A.shape)
        li, ui = (d["step_l"][i - 1], d["step_u"][i - 1]) if i else (l0, u0)
        Ps = sp.diags(c * D) @ P @ sp.diags(D)
        As = sp.diags(E) @ Ai @ sp.diags(D)
        rv = rho_vec(rho, E * np.maximum(li, -INF), E * np.minimum(ui, INF))
        rhs = np.concatenate([SIGMA * st["x"] - c * D * q, st["z"] - st["y"] / rv])
        out.append((sp.csc_matrix(Ps), sp.csc_matrix(As), rv, rhs))
        if i + 1 < steps:
            s.update(l=d["step_l"][i], u=d["step_u"][i])
            s.update(Ax=d["step_Ax"][i], l=d["step_l"][i], u=d["step_u"][i])
    return out


def kkt(Ps, As, rv):
    n = Ps.shape[0]
    Pf = Ps + sp.triu(Ps, 1).T
    return sp.bmat([[Pf + SIGMA * sp.eye(n), As.T], [As, -sp.diags(1.0 / rv)]], format="csc")


def eta(K, x, b):
    """componentwise (Oettli-Prager) backward error max_i |K x - b|_i / (|K| |x| + |b|)_i: the
    normwise one is swamped by the 1/rho diagonal of free and inequality rows"""
    r = np.abs(K @ x - b)
    den = abs(K) @ np.abs(x) + np.abs(b)
    return float(np.max(r / np.maximum(den, 1e-300)))


def run_plan(env, insts):
    from mpc_arpo_project_amd import _lib

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        etas = []
        for Ps, As, rv, rhs in insts:
            As_sorted = sp.csc_matrix(As)
            As_sorted.sort_indices()
            Ps_sorted = sp.csc_matrix(Ps)
            Ps_sorted.sort_indices()
            sol, _ = _lib.schedule_check(Ps_sorted, As_sorted, SIGMA, rv, rhs)
            etas.append(eta(kkt(Ps_sorted, As_sorted, rv), sol, rhs))
        _, _, _, st = _lib.analyze(Ps_sorted, As_sorted)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    e = np.array(etas)
    return dict(steps=st["fwd_steps"] + st["bwd_steps"], lds=st["lds_image_bytes"],
                eta_median=float(np.median(e)), eta_p90=float(np.quantile(e, 0.9)),
                eta_max=float(e.max()), eta_mean_log10=float(np.mean(np.log10(e + 1e-300))))


PLANS = {
    "n20": {
        "tuned": {},
        "r4 default 160/416": dict(MPCQP_CAPM="160", MPCQP_CAPW="416", MPCQP_PAIRED="1"),
        "176/384": dict(MPCQP_CAPM="176", MPCQP_CAPW="384", MPCQP_PAIRED="1"),
        "192/384": dict(MPCQP_CAPM="192", MPCQP_CAPW="384", MPCQP_PAIRED="1"),
        "128/384 (closed loop 0.599)": dict(MPCQP_CAPM="128", MPCQP_CAPW="384", MPCQP_PAIRED="1"),
        "96/320": dict(MPCQP_CAPM="96", MPCQP_CAPW="320", MPCQP_PAIRED="1"),
        "64/256": dict(MPCQP_CAPM="64", MPCQP_CAPW="256", MPCQP_PAIRED="1"),
        "unblocked 1/1": dict(MPCQP_CAPM="1", MPCQP_CAPW="1", MPCQP_PAIRED="1"),
    },
    "n40dv": {
        "tuned": {},
        "128/384": dict(MPCQP_CAPM="128", MPCQP_CAPW="384", MPCQP_PAIRED="1"),
        "96/320": dict(MPCQP_CAPM="96", MPCQP_CAPW="320", MPCQP_PAIRED="1"),
        "unblocked 1/1": dict(MPCQP_CAPM="1", MPCQP_CAPW="1", MPCQP_PAIRED="1"),
    },
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--limit", type=int, default=None)
    a = ap.parse_args()
    os.environ["MPCQP_DIAGNOSTICS"] = "1"
    os.environ.setdefault("MPCQP_LIBRARY", HOST_LIB)
    res = {}
    for tag, fam in (("cl_n20", "n20"), ("cl_noise_n20", "n20"), ("cl_n40dv", "n40dv")):
        insts = instances(tag, a.limit)
        ref = [eta(kkt(Ps, As, rv), spla.spsolve(kkt(Ps, As, rv), rhs), rhs) for Ps, As, rv, rhs in insts]
        res[tag] = {"instances": len(insts), "superlu_eta_median": float(np.median(ref)),
                    "superlu_eta_max": float(np.max(ref))}
        for name, env in PLANS[fam].items():
            try:
                res[tag][name] = run_plan(env, insts)
            except Exception as e:  # a plan the planner refuses
                res[tag][name] = {"error": str(e)}
            print(tag, name, res[tag][name], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
