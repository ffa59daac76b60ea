"""Benchmark: batched warm-started MPC-QP solves in the reference's closed loop, on MI355X.

A "step" is one pass of the hot path over the batch: every chaser's QP (rebuilt on the device from
its new state estimate: configureDynamicConstraints) is re-scaled, re-factored and solved
warm-started by the HIP engine, then the controller select + CW plant advance the chaser
(reference src/trajectorySimulate.py:285-356, noise=None path).  Workload: the radial approach
scenario of reference test/traj_eval_radial.py at horizon N = Nx = 20 (Nc = Nb = 5), planar
4-state / 2-input CW model (n = 121 variables, m = 226 constraints), eps_abs = eps_rel = 1e-4,
B = 65536 chasers per GPU (weak scaling over GPUs: shards of independent chasers, no collective
in the timed region).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--nx 40 --dv]
    (--gpus N > 1 without torchrun: relaunched under torch.distributed.run, one rank per GPU)

Rank 0 prints one JSON line: metric/value/... + roofline (graded on the LDS, the resource the
solve steps run on; HBM and FP64 fractions beside it) + cold (single-shot) rate + cpu_baseline
(Measurement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from mpc_arpo_project_amd import launch  # noqa: E402  (no GPU initialisation at import)

METRIC = "MPC-QP solves/sec @ N=20, 6-state CW, batch=65536; ADMM iters to 1e-4"
HBM_PEAK_GBS = 8000.0      # MI355X spec (MI355X_MICROARCH.md)
LDS_PEAK_GBS = 157286.4    # 256 B/clk/CU (ds_read_b64 rate) x 256 CUs x 2.4 GHz (MICROARCH, LDS)
FP64_PEAK_GFLOPS = 78600.0  # MI355X FP64 vector spec
FAST_ITERS = 1000           # parity: below this the engine and the oracle agree exactly


def bytes_model(n, m, nnzA, nnzL):
    """SURVEY.md 8(d) streaming bytes: per ADMM iteration, per factorization, per-solve I/O."""
    nk = n + m
    b_iter = 8 * (2 * nnzL + nk + 4 * n + 10 * m)
    b_fact = 8 * (nnzA + nnzL + nk)
    b_io = 8 * (2 * m + nnzA + 2 * (n + 2 * m))
    return b_iter, b_fact, b_io


def lds_bytes_per_iter(nfwd, nbwd, n, m):
    """LDS bytes one ADMM iteration of the engine moves (Roofline): every solve step
    is a 64-lane pass of 16 ds_read_b64 (8 operands, 8 vector entries) and 4 ds_add_f64 (a read
    and a write of the LDS array each); the vector passes between the solves touch whole
    register slots: rhs + zero fill 2 (RN + RM), the D^-1 pass 4 (RN + RM), the x / z read-back
    (RN + RM) slot accesses of 512 B.  Factorization, Ruiz passes and termination checks (about
    3 % more at N = 20) are not counted: the figure is a lower bound."""
    need_n, need_m, need_k = -(-n // 64), -(-m // 64), (n + m) // 64 + 1
    slots = next(3 * b for b in (2, 4, 8) if need_n <= b and need_m <= 2 * b and 3 * b >= need_k)
    return (nfwd + nbwd) * 64 * (16 * 8 + 4 * 16) + 7 * slots * 512


def flops_per_solve(iters, n, m, nnzA, nnzL, checks):
    """SURVEY.md 8(d) algorithmic fp64 flops: factorization ~8.7 nnz(L), per iteration
    4 nnz(L) + 10 (n + m) (triangular solves + vector ops), per check ~8.65 nnz(A)
    (= 11.3k + iters 8.7k + 6.2k / check at N = 20)."""
    return 8.7 * nnzL + iters * (4 * nnzL + 10 * (n + m)) + checks * 8.65 * nnzA


def initial_states(B_global, rank, B, seed):
    from mpc_arpo_project_amd import scenarios

    X = scenarios.sample_estimates(B_global, seed=seed)[rank * B:(rank + 1) * B, :4].copy()
    X[:, 2:4] = 0.0  # chasers start at rest, as the reference's x0
    return X


def cgroup_cpus():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else float(q) / float(p)
    except Exception:
        return None


def cpu_baseline(prob, X0, steps, warmup, eps, sample, threads, device):
    """Time the CPU oracle (oracle/, C restatement of OSQP 0.6) on the SAME per-step QPs of a
    bounded sample of chasers: the sample's QP data is recorded from a device closed loop of those
    chasers (identical per chaser to the timed run: shard-invariant), then every solver does the
    reference's per-step update(l, u) + update(Ax) + warm solve.  Only the oracle calls are timed.
    Step 0 is the cold solve (set-up data); its agreement with the engine is reported separately,
    and over the solves both sides finish within FAST_ITERS iterations."""
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
        rec.append((Ax.cpu().numpy(), l.cpu().numpy(), u.cpu().numpy(),
                    r.status.cpu().numpy().copy(), r.iter.cpu().numpy().copy()))
    cl.close()
    solvers = []
    for b in range(S):
        A = sp.csc_matrix((rec[0][0][b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
        s = orc.OracleOSQP()
        s.setup(prob.P, prob.q, A, rec[0][1][b], rec[0][2][b], eps_abs=eps, eps_rel=eps,
                warm_start=True, verbose=False)
        solvers.append(s)
    agree, fast_agree = [], []
    t_cpu = 0.0
    for k in range(warmup + steps):
        if k == 0:
            _, st, it = orc.batch_update_solve(solvers, None, None, None, threads)
        else:
            t0 = time.perf_counter()
            _, st, it = orc.batch_update_solve(solvers, rec[k][0], rec[k][1], rec[k][2], threads)
            dt = time.perf_counter() - t0
            if k >= warmup:
                t_cpu += dt
        same = (st == rec[k][3]) & (it == rec[k][4])
        fast = np.maximum(it, rec[k][4]) <= FAST_ITERS
        agree.append(float(np.mean(st == rec[k][3])))
        fast_agree.append(float(np.mean(same[fast])) if fast.any() else 1.0)
    timed = max(steps if warmup >= 1 else steps - 1, 1)
    return dict(value=S * timed / t_cpu, unit="solves/s", cores=threads, kind="port",
                affinity_cpus=len(os.sched_getaffinity(0)), cgroup_cpu_quota=cgroup_cpus(),
                sample=f"{S} chasers x {timed} warm closed-loop steps (update(l,u)+update(Ax)+solve, "
                       f"eps {eps:g}) after {warmup} untimed steps; {t_cpu:.2f} s on {threads} "
                       f"threads",
                status_agreement_with_gpu=float(np.mean(agree)),
                status_agreement_per_step=[round(a, 5) for a in agree],
                cold_step_status_agreement=agree[0],
                cold_step_exact_agreement_within_1000_iters=fast_agree[0],
                warm_exact_agreement_within_1000_iters=float(np.mean(fast_agree[1:])) if
                len(fast_agree) > 1 else None,
                note="free-running: each oracle solver carries its own warm state, so one "
                     "status flip changes its later starting points; see DESIGN.md, Parity")


def load_traffic(B, nx, split):
    """PMC-measured L2<->fabric bytes per solve launch (tools/pmc_run.sh + tools/pmc_traffic.py),
    with the commit it was measured at"""
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        pj = json.load(open(pmc))
        if pj.get("batch") == B and pj.get("nx") == nx and pj.get("concurrent_shards") == split:
            return pj.get("hbm_bytes_per_launch"), pj.get("commit") or pj.get("kernel_version")
    except Exception:
        pass
    return None, None


def main(argv=None):
    argv = sys.argv if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="chasers per GPU")
    ap.add_argument("--nx", type=int, default=20)
    ap.add_argument("--dv", action="store_true", help="impulsive delta-v input model (BASELINE config 3)")
    ap.add_argument("--eps", type=float, default=1e-4)
    ap.add_argument("--seed", type=int, default=20250328)
    ap.add_argument("--cpu-sample", type=int, default=16384)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads (default: every core in this process's affinity mask)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split", type=int, default=2,
                    help="chaser shards per GPU on concurrent HIP streams (fills one shard's solve "
                         "tail with the other shard's work; 2 measured best, 4 no better than 1)")
    args = ap.parse_args(argv[1:])
    if args.gpus > 1 and not launch.launched():
        # one process per GPU: start torch.distributed.run as a child (nothing has touched the
        # GPU in this process) and exit with its status
        return launch.relaunch(args.gpus, argv)
    import torch

    rank, world, local, device, dist = launch.init("nccl")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but {world} ranks were launched")

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
        cls[-1].enable_tracking(int(sim.T_final / sim.time_stp), *sim.suc_cond)
    torch.cuda.synchronize()
    dims = cls[0].qp.dims()
    sched = cls[0].qp.schedule_info()

    # cold (single-shot) solves: step 0 of the loop solves every chaser from set-up data, no warm
    # start; timed on its own (HIP events on each shard's stream)
    cold_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(S)]
    cold_it = torch.empty(B, dtype=torch.int32, device=device)
    torch.cuda.synchronize()
    tc0 = time.perf_counter()
    for j, c in enumerate(cls):
        cold_ev[j][0].record(c.qp.stream)
        r = c.qp.solve_async()
        cold_ev[j][1].record(c.qp.stream)
        with torch.cuda.stream(c.qp.stream):
            cold_it[cut[j]:cut[j + 1]].copy_(r.iter, non_blocking=True)
        c.step_after_solve(r)
    torch.cuda.synchronize()
    cold_wall = time.perf_counter() - tc0
    for _ in range(max(args.warmup - 1, 0)):
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
    # after the timed region: the per-chaser run summaries (first MPC input, last
    # status, ADMM iterations, i_term, success, final error, fallback steps) of every rank, one
    # all-gather (RCCL over xGMI)
    summ = launch.gather_rows(torch.cat([c.summary() for c in cls]), world * B, rank, world, dist)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # solve-kernel seconds per launch (per shard and step; concurrent shards share the GPU)
    kt = np.array([[a.elapsed_time(b) for a, b in ev[j]] for j in range(S)]) * 1e-3
    it = iters.cpu().numpy()
    ru = rhou.cpu().numpy()
    st = stat.cpu().numpy()
    n, m, nnzA, nnzL = dims["n"], dims["m"], dims["nnzA"], dims["nnzL"]
    b_iter, b_fact, b_io = bytes_model(n, m, nnzA, nnzL)
    lds_iter = lds_bytes_per_iter(sched["fwd_steps"], sched["bwd_steps"], n, m)
    chk = np.ceil(it / 25.0)
    # per launch (shard j, step k): LDS bytes, flops, streaming-model bytes of its instances
    lds_b = np.stack([[float(it[k, cut[j]:cut[j + 1]].sum()) * lds_iter for k in range(K)]
                      for j in range(S)])  # (S, K)
    flops = np.stack([[float(flops_per_solve(it[k, cut[j]:cut[j + 1]], n, m, nnzA, nnzL,
                                             chk[k, cut[j]:cut[j + 1]]).sum()) for k in range(K)]
                      for j in range(S)])
    per_solve = it.astype(np.float64) * b_iter + (1 + ru) * b_fact + b_io  # (K, B)
    stream_b = np.stack([per_solve[:, cut[j]:cut[j + 1]].sum(axis=1) for j in range(S)])
    # rates over the GPU: with S > 1 the shards' launches overlap, so a launch's own duration
    # undercounts; `achieved` = all bytes of the timed region / its wall time (conservative: the
    # gaps between launches count too); the per-launch form (bytes of one launch / its HIP-event
    # duration, x S concurrent launches) is reported beside it
    lds_ach = float(lds_b.sum() / elapsed) / 1e9
    lds_per_launch = float(np.mean(lds_b / kt)) / 1e9
    fl_ach = float(flops.sum() / elapsed) / 1e9
    stream_ach = float(stream_b.sum() / elapsed) / 1e9
    traffic, traffic_at = load_traffic(B, args.nx, S)
    hbm = None
    if traffic:
        ach = traffic * S * K / elapsed / 1e9
        hbm = {"achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
               "bytes_per_launch": traffic, "measured_at": traffic_at,
               "what": "PMC FETCH_SIZE + WRITE_SIZE (L2 <-> fabric, calibrated; tools/pmc_run.sh)"}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return 0
    uniq, cnt = np.unique(st, return_counts=True)
    Sn = summ.cpu().numpy()
    kt_cold = np.array([a.elapsed_time(b) for a, b in cold_ev]) * 1e-3
    ci = cold_it.cpu().numpy()
    metric = METRIC if (args.nx, args.dv) == (20, False) else (
        f"MPC-QP solves/sec @ N={args.nx}{', impulsive delta-v' if args.dv else ''}, CW, "
        f"batch={B}; ADMM iters to {args.eps:g}")
    out = {
        "metric": metric,
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
                        f"slacks + 2 disturbances (n={n}, m={m}), OSQP 0.6 "
                        f"settings with eps_abs=eps_rel={args.eps:g}",
            "batch_per_gpu": B,
            "global_batch": world * B,
            "N": args.nx,
            "parallelism": f"shard{world}" if world > 1 else "single",
            "streams_per_gpu": S,
        },
        "roofline": {
            "bound": "lds",
            "achieved": lds_ach,
            "peak": LDS_PEAK_GBS,
            "unit": "GB/s",
            "frac": lds_ach / LDS_PEAK_GBS,
            "traffic": traffic,
            "kernel": "qp_batch_kernel",
            "kernel_ms_per_launch": float(np.mean(kt) * 1e3),
            "concurrent_shards": S,
            "lds_bytes_per_iter": lds_iter,
            "lds_bytes_per_launch": float(lds_b.mean()),
            "achieved_per_launch": lds_per_launch,
            "why": "one QP per wave with the KKT factor and solve vector in LDS: the solve steps "
                   "are LDS read/atomic passes; HBM carries only per-solve I/O and check reloads",
            "hbm": hbm,
            "fp64": {"achieved": fl_ach, "peak": FP64_PEAK_GFLOPS, "unit": "GFLOP/s",
                     "frac": fl_ach / FP64_PEAK_GFLOPS},
            "streaming_model": {"achieved": stream_ach, "unit": "GB/s",
                                "frac_of_hbm_peak": stream_ach / HBM_PEAK_GBS,
                                "bytes_model": {"per_iter": b_iter, "per_factor": b_fact,
                                                "per_solve_io": b_io},
                                "note": "SURVEY 8(d) accounting (factor and iterates streamed "
                                        "every iteration); they stay in LDS/VGPRs instead"},
        },
        "cold": {"value": world * B / cold_wall, "unit": "solves/s", "wall_ms": cold_wall * 1e3,
                 "kernel_ms_per_launch": float(kt_cold.mean() * 1e3),
                 "admm_iters_mean": float(ci.mean()),
                 "what": "step 0: every chaser solved once from its set-up data, no warm start"},
        "admm_iters": {"mean": float(it.mean()), "median": float(np.median(it)),
                       "p90": float(np.percentile(it, 90)), "max": int(it.max())},
        "status_counts": {str(int(a)): int(c) for a, c in zip(uniq, cnt)},
        "schedule": sched,
        "summary_gather": {"rows": int(Sn.shape[0]), "fields": list(cls[0].SUMMARY_FIELDS),
                           "bytes": int(Sn.nbytes),
                           "mean_admm_iters_per_chaser": float(Sn[:, 3].mean())},
    }
    if world == 1 and not args.no_cpu_baseline:
        try:
            # every core this process may run on: the affinity mask, capped by the cgroup CPU
            # quota when one is set (the GPU box grants 16 CPUs of a 256-thread host: 256 threads
            # on a 16-CPU quota measured 2.3x slower than 16)
            aff = len(os.sched_getaffinity(0))
            quota = cgroup_cpus()
            thr = args.cpu_threads or (min(aff, int(quota)) if quota and quota >= 1 else aff)
            out["cpu_baseline"] = cpu_baseline(prob, X0, K, args.warmup, args.eps, args.cpu_sample,
                                               thr, device)
        except Exception as e:  # report, never fake
            out["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    for c in cls:
        c.close()
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
