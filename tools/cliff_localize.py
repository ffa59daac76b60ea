"""Where do the high-register diagnostic builds (High-register builds) first compute
something different?  Runs 64 instances of the batch_n20 fixture through the library named by
MPCQP_LIBRARY under settings that cut the solve short or switch phases off, and saves every output
(status, iterations, x, y, scaled warm state) to an npz; `compare a.npz b.npz` prints, per setting,
whether two builds agree bitwise and the first differing array.

usage: MPCQP_LIBRARY=... python tools/cliff_localize.py run out.npz
       python tools/cliff_localize.py compare a.npz b.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

SETTINGS = {
    "iter1": dict(max_iter=1, check_termination=0, adaptive_rho=0),
    "iter1_noscale": dict(max_iter=1, check_termination=0, adaptive_rho=0, scaling=0),
    "iter2": dict(max_iter=2, check_termination=0, adaptive_rho=0),
    "iter25": dict(max_iter=25, adaptive_rho=0),
    "iter200": dict(max_iter=200),
    "full": dict(),
    # B > the persistent grid (1,024 waves): waves take a second, third ... instance
    "full_b4096": dict(B=4096),
    "iter1_b4096": dict(B=4096, max_iter=1, check_termination=0, adaptive_rho=0),
    # a warm second solve of the same data (has_state = 1) at B = 64
    "warm": dict(warm=True),
}


def run(out):
    from conftest import load_golden, problem
    from mpc_arpo_project_amd.engine import BatchQP

    prob = problem(20, False)
    d = load_golden("batch_n20")
    res = {}
    nf = d["Ax"].shape[0]
    for name, st in SETTINGS.items():
        st = dict(st)
        B, warm = st.pop("B", 64), st.pop("warm", False)
        idx = np.arange(B) % nf
        qp = BatchQP(prob.P, prob.A, batch=B, eps_abs=1e-4, eps_rel=1e-4, **st)
        qp.set_data(q=prob.q, Ax=d["Ax"][idx], l=d["l"][idx], u=d["u"][idx])
        r = qp.solve()
        if warm:
            r = qp.solve()
        res[f"{name}.status"] = r.status.cpu().numpy()
        res[f"{name}.iter"] = r.iter.cpu().numpy()
        res[f"{name}.x"] = r.x.cpu().numpy()
        res[f"{name}.y"] = r.y.cpu().numpy()
        for k, v in qp.get_state().items():
            res[f"{name}.state_{k}"] = v.cpu().numpy()
        qp.close()
    np.savez(out, **res)


def self_consistent(path):
    """B = 4096 runs repeat the 64 fixture instances 64 times: every copy must match the first"""
    Z = np.load(path)
    for k in Z.files:
        if "_b4096." not in k or Z[k].ndim == 0:
            continue
        x = Z[k].reshape(64, 64, *Z[k].shape[1:])
        same = np.array([np.array_equal(x[c], x[0], equal_nan=True) for c in range(64)])
        print(f"{os.path.basename(path)} {k}: copies equal to the first {same.sum()} / 64")


def compare(a, b):
    self_consistent(a)
    self_consistent(b)
    A, Bz = np.load(a), np.load(b)
    for name in SETTINGS:
        keys = [k for k in A.files if k.startswith(name + ".")]
        diff = [k for k in keys if not np.array_equal(A[k], Bz[k], equal_nan=True)]
        if not diff:
            print(f"{name}: bitwise equal ({len(keys)} arrays)")
            continue
        k = diff[0]
        x, y = A[k].astype(float), Bz[k].astype(float)
        rows = np.unique(np.nonzero(~((x == y) | (np.isnan(x) & np.isnan(y))))[0])
        print(f"{name}: differ in {diff}; first {k}: {len(rows)} of {x.shape[0]} instances, "
              f"max |d| {np.nanmax(np.abs(x - y)):.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
