"""Benchmark: batched warm-started MPC-QP solves in the reference's closed loop, on MI355X.

A "step" is one pass of the hot path over the batch: every chaser's QP (rebuilt on the device from
its new state estimate: configureDynamicConstraints) is re-scaled, re-factored and solved
warm-started by the HIP engine, then the controller select + CW plant advance the chaser
(reference src/trajectorySimulate.py:285-356, noise=None path).  Workload: the radial approach
scenario of reference test/traj_eval_radial.py at horizon N = Nx = 20 (Nc = Nb = 5), planar
4-state / 2-input CW model (n = 121 variables, m = 226 constraints), eps_abs = eps_rel = 1e-4,
B = 65536 chasers per GPU (weak scaling over GPUs: shards of independent chasers, no collective
in the timed region).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line (metric/value/... + roofline + cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "MPC-QP solves/sec @ N=20, 6-state CW, batch=65536; ADMM iters to 1e-4"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)


def bytes_model(n, m, nnzA, nnzL):
    """SURVEY.md 8(d) algorithmic bytes: per ADMM iteration, per factorization, per-solve I/O."""
    nk = n + m
    b_iter = 8 * (2 * nnzL + nk + 4 * n + 10 * m)
    b_fact = 8 * (nnzA + nnzL + nk)
    b_io = 8 * (2 * m + nnzA + 2 * (n + 2 * m))
    return b_iter, b_fact, b_io


def initial_states(B_global, rank, B, seed):
    from mpc_arpo_project_amd import scenarios

    X = scenarios.sample_estimates(B_global, seed=seed)[rank * B:(rank + 1) * B, :4].copy()
    X[:, 2:4] = 0.0  # chasers start at rest, as the reference's x0
    return X


def cpu_baseline(prob, X0, steps, warmup, eps, sample, threads, device):
    """Time the CPU oracle (oracle/, C restatement of OSQP 0.6) on the SAME per-step QPs of a
    bounded sample of chasers: the sample's QP data is recorded from a device closed loop of those
    chasers (identical per chaser to the timed run: shard-invariant), then every solver does the
    reference's per-step update(l, u) + update(Ax) + warm solve.  Only the oracle calls are timed."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    import scipy.sparse as sp
    from mpc_arpo_project_amd.closed_loop import BatchClosedLoop

    S = min(sample, X0.shape[0])
    cl = BatchClosedLoop(prob, X0[:S], device=device, eps_abs=eps, eps_rel=eps)
    rec = []
    for k in range(warmup + steps):
        Ax, l, u = cl.qp.copy_data()
        r = cl.step()
        rec.append((Ax.cpu().numpy(), l.cpu().numpy(), u.cpu().numpy(), r.status.cpu().numpy().copy()))
    cl.close()
    solvers = []
    for b in range(S):
        A = sp.csc_matrix((rec[0][0][b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
        s = orc.OracleOSQP()
        s.setup(prob.P, prob.q, A, rec[0][1][b], rec[0][2][b], eps_abs=eps, eps_rel=eps,
                warm_start=True, verbose=False)
        solvers.append(s)
    agree = []
    # step 0 solves straight after set-up; later steps update then solve
    t_cpu = 0.0
    for k in range(warmup + steps):
        if k == 0:
            _, st, _ = orc.batch_update_solve(solvers, None, None, None, threads)
        else:
            t0 = time.perf_counter()
            _, st, _ = orc.batch_update_solve(solvers, rec[k][0], rec[k][1], rec[k][2], threads)
            dt = time.perf_counter() - t0
            if k >= warmup:
                t_cpu += dt
        agree.append(float(np.mean(st == rec[k][3])))
    timed = max(steps if warmup >= 1 else steps - 1, 1)
    return dict(value=S * timed / t_cpu, unit="solves/s", cores=threads, kind="port",
                sample=f"{S} chasers x {timed} warm closed-loop steps (update(l,u)+update(Ax)+solve, "
                       f"eps {eps:g}) after {warmup} untimed steps; {t_cpu:.2f} s on {threads} "
                       f"threads",
                status_agreement_with_gpu=float(np.mean(agree)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="chasers per GPU")
    ap.add_argument("--nx", type=int, default=20)
    ap.add_argument("--dv", action="store_true", help="impulsive delta-v input model (BASELINE config 3)")
    ap.add_argument("--eps", type=float, default=1e-4)
    ap.add_argument("--seed", type=int, default=20250328)
    ap.add_argument("--cpu-sample", type=int, default=16384)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split", type=int, default=2,
                    help="chaser shards per GPU on concurrent HIP streams (fills one shard's solve "
                         "tail with the other shard's work; 2 measured best, 4 no better than 1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=device)

    from mpc_arpo_project_amd import qp_model, scenarios
    from mpc_arpo_project_amd.closed_loop import BatchClosedLoop

    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=args.nx, isDeltaV=args.dv)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    B = args.batch
    X0 = initial_states(world * B, rank, B, args.seed)
    S = max(1, min(args.split, B))
    # S shards of the chasers, each a closed loop on its own HIP stream; shard j holds global chaser
    # ids [rank*B + cut[j], rank*B + cut[j+1]), so results do not depend on S
    cut = [B * j // S for j in range(S + 1)]
    cls = []
    for j in range(S):
        st_j = torch.cuda.Stream(device=device) if S > 1 else None
        cls.append(BatchClosedLoop(prob, X0[cut[j]:cut[j + 1]], device=device, eps_abs=args.eps,
                                   eps_rel=args.eps, stream=st_j, id_offset=rank * B + cut[j]))
    torch.cuda.synchronize()
    cl = cls[0]
    dims = cl.qp.dims()
    sched = cl.qp.schedule_info()

    for _ in range(args.warmup):
        for c in cls:
            c.step()
    K = args.steps
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
          for _ in range(S)]
    iters = torch.empty(K, B, dtype=torch.int32, device=device)
    rhou = torch.empty(K, B, dtype=torch.int32, device=device)
    stat = torch.empty(K, B, dtype=torch.int32, device=device)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        for j, c in enumerate(cls):
            stream = c.qp.stream
            ev[j][k][0].record(stream)
            r = c.qp.solve_async()
            ev[j][k][1].record(stream)
            with torch.cuda.stream(stream):
                iters[k, cut[j]:cut[j + 1]].copy_(r.iter, non_blocking=True)
                rhou[k, cut[j]:cut[j + 1]].copy_(r.rho_updates, non_blocking=True)
                stat[k, cut[j]:cut[j + 1]].copy_(r.status, non_blocking=True)
            c.step_after_solve(r)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the only collective: gather every shard's final chaser states (outside the timed region)
        x_all = torch.cat([c.x_true for c in cls])
        gathered = [torch.empty_like(x_all) for _ in range(world)]
        dist.all_gather(gathered, x_all)

    # solve-kernel seconds per launch (per shard and step; concurrent shards share the GPU)
    kt = np.array([[a.elapsed_time(b) for a, b in ev[j]] for j in range(S)]) * 1e-3
    it = iters.cpu().numpy()
    ru = rhou.cpu().numpy()
    st = stat.cpu().numpy()
    b_iter, b_fact, b_io = bytes_model(dims["n"], dims["m"], dims["nnzA"], dims["nnzL"])
    per_solve = it.astype(np.float64) * b_iter + (1 + ru) * b_fact + b_io  # (K, B)
    if S == 1:
        achieved = float(np.mean(per_solve.sum(axis=1) / kt[0])) / 1e9
    else:  # overlapping launches: all algorithmic bytes over the wall time of the timed region
        achieved = float(per_solve.sum() / elapsed) / 1e9
    # the per-launch form (a shard's step bytes over that launch's own duration), which undercounts
    # when launches overlap: reported beside `achieved` for transparency
    shard_bytes = np.stack([per_solve[:, cut[j]:cut[j + 1]].sum(axis=1) for j in range(S)])  # (S, K)
    achieved_per_launch = float(np.mean(shard_bytes / kt)) / 1e9
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            if pj.get("batch") == B and pj.get("nx") == args.nx:
                traffic = pj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    uniq, cnt = np.unique(st, return_counts=True)
    out = {
        "metric": METRIC,
        "value": world * B * K / elapsed,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded chaser states in the LOS cone; radial scenario constants of "
                "reference test/traj_eval_radial.py)",
        "config": {
            "workload": f"warm closed-loop MPC-QP solves (rescale + LDL' refactor + ADMM), radial "
                        f"CW scenario, N=Nx={args.nx}, Nc=Nb=5, planar 4-state/2-input "
                        f"{'impulsive delta-v ' if args.dv else ''}model + 5 "
                        f"slacks + 2 disturbances (n={dims['n']}, m={dims['m']}), OSQP 0.6 "
                        f"settings with eps_abs=eps_rel={args.eps:g}",
            "batch_per_gpu": B,
            "global_batch": world * B,
            "N": args.nx,
            "parallelism": f"shard{world}" if world > 1 else "single",
            "streams_per_gpu": S,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "achieved_per_launch": achieved_per_launch,
            "traffic": traffic,
            "kernel": "qp_batch_kernel",
            "kernel_ms_per_launch": float(np.mean(kt) * 1e3),
            "concurrent_shards": S,
            "bytes_model": {"per_iter": b_iter, "per_factor": b_fact, "per_solve_io": b_io},
        },
        "admm_iters": {"mean": float(it.mean()), "median": float(np.median(it)),
                       "p90": float(np.percentile(it, 90)), "max": int(it.max())},
        "status_counts": {str(int(a)): int(c) for a, c in zip(uniq, cnt)},
        "schedule": sched,
    }
    if world == 1 and not args.no_cpu_baseline:
        try:
            thr = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
            out["cpu_baseline"] = cpu_baseline(prob, X0, K, args.warmup, args.eps, args.cpu_sample,
                                               thr, device)
        except Exception as e:  # report, never fake
            out["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
