"""Parity of the HIP engine with the CPU oracle at bench scale (GPU box; diagnostic tool).

    python tools/parity_scale.py warm   [--batch 16384] [--steps 25] [--eps 1e-4] [--threads T]
    python tools/parity_scale.py growth [--batch 2048]  [--nx 20] [--dv]
    python tools/parity_scale.py cold   [--nx 20] [--dv]        (vs tests/golden/cold_b65536_*.npz)

warm   -- the bench's closed loop (radial scenario, N = 20) on the GPU; every step's QP data and the
          engine's warm state are recorded, then the oracle replays the same per-step
          update(l, u) + update(Ax) + solve twice:
            free:  each oracle solver carries its own warm state (the bench's cpu_baseline, the
                   reference's own semantics, reference src/trajectorySimulate.py:296-348);
            sync:  before every step the oracle solver is given the engine's warm state
                   (mpcqp_get_state -> oqp_set_state), so each solve starts bit-identical and
                   a disagreement is the single solve's own sensitivity.
          Reports per-step status / iteration agreement of both modes, the first step at which
          each chaser's free run diverges, the sync-mode flips with their residuals, and the u0
          differences.
growth -- cold solves with termination checks and rho adaptation off, stopped after k
          iterations: max relative difference of the GPU and oracle iterates vs k (how rounding
          differences grow through the ADMM recursion).
cold   -- cold B = 65,536 solves against the committed oracle fixtures.
Prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle as orc  # noqa: E402  (the checker)
from mpc_arpo_project_amd import qp_model, scenarios  # noqa: E402
from mpc_arpo_project_amd.closed_loop import BatchClosedLoop  # noqa: E402
from mpc_arpo_project_amd.engine import BatchQP  # noqa: E402


def threads_default():
    return len(os.sched_getaffinity(0))


def problem(nx, dv):
    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=nx, isDeltaV=dv)
    return qp_model.build_problem(sim, mpc, fail, deb)


def status_table(a, b):
    pairs = {}
    for x, y in zip(a.tolist(), b.tolist()):
        if x != y:
            pairs[f"{x}->{y}"] = pairs.get(f"{x}->{y}", 0) + 1
    return pairs


def warm(args):
    import scipy.sparse as sp

    prob = problem(args.nx, args.dv)
    B, K, eps = args.batch, args.steps, args.eps
    X = scenarios.sample_estimates(B, seed=20250328)[:, :4].copy()
    X[:, 2:4] = 0.0
    cl = BatchClosedLoop(prob, X, device="cuda", eps_abs=eps, eps_rel=eps)
    rec = []
    t0 = time.time()
    for k in range(K):
        Ax, l, u = cl.qp.copy_data()
        stt = cl.qp.get_state()
        r = cl.step()
        torch.cuda.synchronize()
        rec.append(dict(Ax=Ax.cpu().numpy(), l=l.cpu().numpy(), u=u.cpu().numpy(),
                        xs=stt["x"].cpu().numpy(), zs=stt["z"].cpu().numpy(),
                        ys=stt["y"].cpu().numpy(), rho=stt["rho"].cpu().numpy(),
                        st=r.status.cpu().numpy().copy(), it=r.iter.cpu().numpy().copy(),
                        u0=r.x[:, prob.u0_slice].cpu().numpy().copy(),
                        pr=r.pri_res.cpu().numpy().copy(), dr=r.dua_res.cpu().numpy().copy()))
    cl.close()
    t_gpu = time.time() - t0

    def make_solvers():
        out = []
        for b in range(B):
            A = sp.csc_matrix((rec[0]["Ax"][b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
            s = orc.OracleOSQP()
            s.setup(prob.P, prob.q, A, rec[0]["l"][b], rec[0]["u"][b], eps_abs=eps, eps_rel=eps,
                    warm_start=True, verbose=False)
            out.append(s)
        return out

    T = args.threads or threads_default()
    res = {}
    for mode in ("free", "sync"):
        solvers = make_solvers()
        per = []
        first_div = np.full(B, -1)
        t0 = time.time()
        for k in range(K):
            g = rec[k]
            if k == 0:
                xo, st, it = orc.batch_update_solve(solvers, None, None, None, T)
            else:
                if mode == "sync":
                    orc.batch_set_state(solvers, g["xs"], g["zs"], g["ys"], g["rho"])
                xo, st, it = orc.batch_update_solve(solvers, g["Ax"], g["l"], g["u"], T)
            u0o = xo[:, prob.u0_slice]
            same_st = st == g["st"]
            same_it = it == g["it"]
            both = (st == 1) & (g["st"] == 1)
            du = np.abs(u0o - g["u0"]).max(axis=1)
            du_same = du[both & same_it]
            div = (~same_st | ~same_it) & (first_div < 0)
            first_div[div] = k
            flips = np.nonzero(~same_st)[0]
            per.append(dict(
                step=k, status_agree=float(same_st.mean()), iter_agree=float(same_it.mean()),
                n_status_flip=int((~same_st).sum()), n_iter_diff=int((~same_it).sum()),
                flips=status_table(g["st"], st),
                max_du0_both_solved=float(du[both].max()) if both.any() else None,
                max_du0_same_iter=float(du_same.max()) if du_same.size else None,
                median_du0_same_iter=float(np.median(du_same)) if du_same.size else None,
                max_du0_diff_iter=float(du[both & ~same_it].max()) if (both & ~same_it).any() else None,
                flip_examples=[dict(b=int(b), gpu=[int(g["st"][b]), int(g["it"][b])],
                                    oracle=[int(st[b]), int(it[b])],
                                    gpu_res=[float(g["pr"][b]), float(g["dr"][b])])
                               for b in flips[:6]]))
        res[mode] = dict(
            seconds=time.time() - t0, steps=per,
            status_agree_mean=float(np.mean([p["status_agree"] for p in per])),
            iter_agree_mean=float(np.mean([p["iter_agree"] for p in per])),
            chasers_ever_diverged=float((first_div >= 0).mean()),
            first_divergence_hist={int(k): int(c) for k, c in
                                   zip(*np.unique(first_div[first_div >= 0], return_counts=True))})
        del solvers
    return dict(mode="warm", batch=B, steps=K, eps=eps, nx=args.nx, dv=args.dv, threads=T,
                gpu_seconds=t_gpu, **res)


def growth(args):
    prob = problem(args.nx, args.dv)
    B = args.batch
    Ax, l, u = qp_model.configure_batch(prob, scenarios.sample_estimates(B))
    T = args.threads or threads_default()
    out = []
    for adaptive in (0, 1):
        for k in (1, 2, 5, 10, 25, 50, 100, 101, 200, 400, 800, 1600):
            st = dict(max_iter=k, check_termination=0, adaptive_rho=adaptive, eps_abs=1e-4,
                      eps_rel=1e-4)
            qp = BatchQP(prob.P, prob.A, batch=B, device="cuda", **st)
            qp.set_data(q=prob.q, Ax=Ax, l=l, u=u)
            r = qp.solve()
            xg = r.x.cpu().numpy()
            qp.close()
            xo, _, so, _ = orc.batch_solve(prob.P, prob.q, prob.A, Ax, l, u, nthreads=T, **st)
            ok = np.isfinite(xg).all(axis=1) & np.isfinite(xo).all(axis=1)
            rel = np.abs(xg[ok] - xo[ok]).max(axis=1) / np.maximum(np.abs(xo[ok]).max(axis=1), 1e-300)
            out.append(dict(adaptive_rho=adaptive, iters=k, n=int(ok.sum()),
                            max_rel=float(rel.max()), median_rel=float(np.median(rel)),
                            p99_rel=float(np.percentile(rel, 99))))
    return dict(mode="growth", batch=B, nx=args.nx, dv=args.dv, rows=out)


def cold(args):
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_cold_batch as gcb

    tag = "n40dv" if args.dv else "n20"
    fx = np.load(os.path.join(REPO, "tests", "golden", f"cold_b65536_{tag}.npz"))
    prob, X, Ax, l, u = gcb.inputs(tag)
    assert gcb.digest(Ax, l, u) == str(fx["sha256"]), "inputs differ from the fixture's"
    eps = float(fx["eps"])
    qp = BatchQP(prob.P, prob.A, batch=gcb.B, device="cuda", eps_abs=eps, eps_rel=eps)
    qp.set_data(q=prob.q, Ax=Ax, l=l, u=u)
    torch.cuda.synchronize()
    t0 = time.time()
    r = qp.solve()
    dt = time.time() - t0
    st, it = r.status.cpu().numpy(), r.iter.cpu().numpy()
    u0 = r.x[:, prob.u0_slice].cpu().numpy()
    so, io, uo = fx["status"].astype(np.int32), fx["iter"].astype(np.int32), fx["u0"]
    both = (st == 1) & (so == 1)
    same = both & (it == io)
    du = np.abs(u0 - uo).max(axis=1)
    return dict(mode="cold", tag=tag, batch=gcb.B, seconds=dt, solves_per_s=gcb.B / dt,
                status_agree=float((st == so).mean()), iter_agree=float((it == io).mean()),
                flips=status_table(so, st), n_iter_diff=int((it != io).sum()),
                iter_diff_examples=[[int(b), int(io[b]), int(it[b])] for b in np.nonzero(it != io)[0][:10]],
                max_du0_both_solved=float(du[both].max()),
                max_du0_same_iter=float(du[same].max()), mean_iter=float(it.mean()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("warm", "growth", "cold"))
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--eps", type=float, default=1e-4)
    ap.add_argument("--nx", type=int, default=20)
    ap.add_argument("--dv", action="store_true")
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    if a.mode == "warm":
        a.batch = a.batch or 16384
        out = warm(a)
    elif a.mode == "growth":
        a.batch = a.batch or 2048
        out = growth(a)
    else:
        out = cold(a)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
