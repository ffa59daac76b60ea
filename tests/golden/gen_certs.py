"""Generates tests/golden/cert256_{n20,n40dv}.npz: KKT-certified optimal solutions of >= 256 solved
instances per configuration, the anchor of the north-star tolerance test
(||u0 - u0*||_inf < 1e-5 at eps_abs = eps_rel = 1e-6, tests/test_gpu_scale_parity.py).

Inputs: estimates from `scenarios.sample_estimates(CAND, seed=SEED)` pushed through
`qp_model.configure_batch` (the restatement of the reference's configureDynamicConstraints,
reference src/simhelpers.py:11-140, bit-exact against the reference in tests/test_qp_model.py); a
SHA-256 of the inputs is stored so a test proves it rebuilt the same QPs.

Solutions: the oracle (OSQP 0.6 restatement, test infrastructure) at eps 1e-10 with polish, then a
KKT certificate computed here with numpy / scipy.sparse on the UNSCALED data:
  prim  = max violation of l <= A x <= u            / max(1, |A x|_inf)
  stat  = |P x + q + A' y|_inf                       / max(1, |P x|, |q|, |A' y|)
  comp  = max over rows with |y| > 1e-6 |y|_inf of the distance of A x to the bound y's sign
          selects                                    / max(1, |A x|_inf)
An instance is kept when the oracle reports 'solved', polish succeeded and all three are <= 1e-9.
(Instances the oracle finds primal infeasible are not certified here.)

    python tests/golden/gen_certs.py [procs]          (~3 min on 8 cores)
"""
import hashlib
import os
import sys
from multiprocessing import Pool

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

SEED = 424242
CAND = 400
TOL = 1e-9
CONFIGS = {"n20": dict(Nx=20, isDeltaV=False), "n40dv": dict(Nx=40, isDeltaV=True)}


def inputs(tag):
    from mpc_arpo_project_amd import qp_model, scenarios

    sim, mpc, fail, deb = scenarios.radial_scenario(**CONFIGS[tag])
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    X = scenarios.sample_estimates(CAND, seed=SEED)
    Ax, l, u = qp_model.configure_batch(prob, X)
    return prob, X, Ax, l, u


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def certify(P, q, A, l, u, x, y):
    Ax = A @ x
    scale = max(1.0, float(np.max(np.abs(Ax))))
    lo = np.maximum(l, -1e30)
    hi = np.minimum(u, 1e30)
    prim = max(float(np.max(lo - Ax)), float(np.max(Ax - hi)), 0.0) / scale
    Px, Aty = P @ x, A.T @ y
    g = Px + q + Aty
    gs = max(float(np.max(np.abs(Px))), float(np.max(np.abs(q))), float(np.max(np.abs(Aty))), 1.0)
    stat = float(np.max(np.abs(g))) / gs
    thr = 1e-6 * max(float(np.max(np.abs(y))), 1e-300)
    comp_up = float(np.max(np.where(y > thr, np.abs(hi - Ax), 0.0)))
    comp_lo = float(np.max(np.where(y < -thr, np.abs(Ax - lo), 0.0)))
    return prim, stat, max(comp_up, comp_lo) / scale


_W = {}


def _init(tag):
    _W["data"] = inputs(tag)


def _one(b):
    import oracle as orc

    prob, X, Axb, lb, ub = _W["data"]
    A = sp.csc_matrix((Axb[b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
    P = sp.csc_matrix(prob.P)
    Pfull = P + sp.triu(P, 1).T if sp.tril(P, -1).nnz == 0 else P
    s = orc.OracleOSQP()
    s.setup(prob.P, prob.q, A, lb[b], ub[b], eps_abs=1e-10, eps_rel=1e-10, max_iter=400000,
            polish=True, polish_refine_iter=20, warm_start=True, verbose=False)
    r = s.solve()
    if r.info.status_val != 1 or r.info.status_polish != 1:
        return b, r.info.status_val, r.info.status_polish, None
    c = certify(Pfull, prob.q, A, lb[b], ub[b], r.x, r.y)
    return b, r.info.status_val, r.info.status_polish, (r.x, r.y, r.info.obj_val, c)


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    for tag in CONFIGS:
        prob, X, Ax, l, u = inputs(tag)
        with Pool(procs, initializer=_init, initargs=(tag,)) as pool:
            res = pool.map(_one, range(CAND), chunksize=4)
        keep = [(b, v) for b, st, pol, v in res if v is not None and max(v[3]) <= TOL]
        stats = {}
        for b, st, pol, v in res:
            k = f"status {st} polish {pol}" + ("" if v is None else (" certified" if max(v[3]) <= TOL else " cert>tol"))
            stats[k] = stats.get(k, 0) + 1
        idx = np.array([b for b, _ in keep], dtype=np.int32)
        xs = np.array([v[0] for _, v in keep])
        np.savez_compressed(os.path.join(HERE, f"cert256_{tag}.npz"), idx=idx, x=xs,
                            y=np.array([v[1] for _, v in keep]),
                            obj=np.array([v[2] for _, v in keep]),
                            cert=np.array([v[3] for _, v in keep]),
                            u0=xs[:, prob.u0_slice], seed=SEED, cand=CAND,
                            sha256=np.array(digest(Ax, l, u)))
        print(tag, "certified", len(idx), stats, "max cert", float(np.max([max(v[3]) for _, v in keep])),
              flush=True)


if __name__ == "__main__":
    main()
