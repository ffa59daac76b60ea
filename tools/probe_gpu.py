"""Quick GPU probe: parity vs oracle on fixture instances + a throughput sample."""
import os, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as orc
from mpc_arpo_project_amd import qp_model, scenarios
from mpc_arpo_project_amd.engine import BatchQP

def run(Nx, dv, eps, B_time):
    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=Nx, isDeltaV=dv)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    fx = np.load(os.path.join(REPO, "tests/golden/batch_n%s.npz" % ("20" if Nx == 20 else "40dv")))
    Ax, l, u = fx["Ax"], fx["l"], fx["u"]
    B = Ax.shape[0]
    st = dict(eps_abs=eps, eps_rel=eps)
    qp = BatchQP(prob.P, prob.A, batch=B, **st)
    print("dims", qp.dims(), "sched", qp.schedule_info(), flush=True)
    qp.set_data(q=prob.q, Ax=Ax, l=l, u=u)
    t0 = time.time(); r = qp.solve(); t1 = time.time()
    xo, yo, so, io = orc.batch_solve(prob.P, prob.q, prob.A, Ax, l, u, nthreads=8, **st)
    sg, ig = r.status.cpu().numpy(), r.iter.cpu().numpy()
    xg = r.x.cpu().numpy()
    sl = prob.u0_slice
    ok = (sg == so)
    print(f"Nx={Nx}: status match {ok.sum()}/{B}; iter match {(ig==io).sum()}/{B}; gpu {t1-t0:.3f}s")
    print(" gpu status", np.unique(sg, return_counts=True), " oracle", np.unique(so, return_counts=True))
    both = ok & (so == 1)
    if both.any():
        e = np.abs(xg[both][:, sl] - xo[both][:, sl]).max()
        ex = np.nanmax(np.abs(xg[both] - xo[both]) / (1 + np.abs(xo[both])))
        print(f" solved both: {both.sum()}  max|u0 diff| {e:.3e}  max rel x diff {ex:.3e}")
    bad = np.nonzero(~ok)[0][:5]
    for b in bad: print("  mismatch", b, sg[b], so[b], ig[b], io[b])
    print(" iters gpu", ig[:16], "\n iters orc", io[:16], flush=True)
    # throughput sample
    X = scenarios.sample_estimates(B_time, seed=1); X[:, 2:4] = 0.0
    Ax2, l2, u2 = qp_model.configure_batch(prob, X)
    qp2 = BatchQP(prob.P, prob.A, batch=B_time, **st)
    qp2.set_data(q=prob.q, Ax=Ax2, l=l2, u=u2)
    r2 = qp2.solve()
    torch.cuda.synchronize(); t0 = time.time(); r2 = qp2.solve_async(); torch.cuda.synchronize(); t1 = time.time()
    it2 = r2.iter.cpu().numpy(); s2 = r2.status.cpu().numpy()
    print(f" B={B_time} warm re-solve: {t1-t0:.4f}s -> {B_time/(t1-t0):.0f} solves/s; iters mean {it2.mean():.1f} med {np.median(it2)} max {it2.max()}; status {np.unique(s2, return_counts=True)}", flush=True)

run(20, False, 1e-4, int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
run(40, True, 1e-4, int(sys.argv[1]) if len(sys.argv) > 1 else 4096)

def iter_cost(Nx, dv):
    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=Nx, isDeltaV=dv)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    for iters in (0, 200):
        for B in (1, 2048):
            X = scenarios.sample_estimates(B, seed=3); X[:, 2:4] = 0.0
            Ax, l, u = qp_model.configure_batch(prob, X)
            qp = BatchQP(prob.P, prob.A, batch=B, check_termination=0, adaptive_rho=0, max_iter=max(iters, 1), warm_start=False)
            qp.set_data(q=prob.q, Ax=Ax, l=l, u=u)
            qp.solve()
            ts = []
            for _ in range(3):
                torch.cuda.synchronize(); t0 = time.time(); qp.solve_async(); torch.cuda.synchronize(); ts.append(time.time() - t0)
            print(f"Nx={Nx} B={B} max_iter={max(iters,1)}: {min(ts)*1e3:.3f} ms  sched={qp.schedule_info()}", flush=True)

iter_cost(20, False)
