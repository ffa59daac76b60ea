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
    python bench.py --continuous     (BASELINE config 4: trajectorySimulateC's loop, see below)
    (--gpus N > 1 without torchrun: relaunched under torch.distributed.run, one rank per GPU)

Rank 0 prints one JSON line: metric/value/... + roofline (graded on the LDS, the resource the
solve steps run on; HBM and FP64 fractions beside it) + cold (single-shot) rate + cpu_baseline
+ four legs measured in the same run, each with its own roofline: config3 (N = 40 impulsive
delta-v, BASELINE config 3) and n40_accel (N = 40 continuous acceleration, the horizon of every
reference script), both at the headline's window, config2 (BASELINE config 2: B = 1,024 at N = 20,
one launch) and config4 (the continuous-time nonlinear loop, BASELINE config 4, --cont-steps
sample periods).  `value` counts the solves the engine ran: chasers that terminated
(reference src/trajectorySimulate.py:288-293) are skipped by the solver and not counted.
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


def lds_bytes_per_iter(nfwd, nbwd, n, m, atomics_per_step):
    """LDS bytes one ADMM iteration of the engine moves (Roofline): every solve step
    is a 64-lane pass of 16 ds_read_b64 (8 operands, 8 vector entries) and `atomics_per_step`
    ds_add_f64 (a read and a write of the LDS array each: 16 B per lane; 3 on paired steps, where
    a lane sums its segments 0 + 1 into one target, 4 otherwise); the vector passes between the
    solves touch whole register slots: rhs + zero fill 2 (RN + RM), the D^-1 pass 4 (RN + RM),
    the x / z read-back (RN + RM) slot accesses of 512 B.  Factorization, Ruiz passes and
    termination checks are not counted: the figure is a lower bound."""
    need_n, need_m, need_k = -(-n // 64), -(-m // 64), (n + m) // 64 + 1
    slots = next(3 * b for b in (2, 4, 8) if need_n <= b and need_m <= 2 * b and 3 * b >= need_k)
    return (nfwd + nbwd) * 64 * (16 * 8 + atomics_per_step * 16) + 7 * slots * 512


LDS_CLK_GHZ = 2.4          # the LDS array serves one cycle per clock per CU (MICROARCH, LDS)


def lds_cycles_per_iter(nfwd, nbwd, n, m, atomics_per_step):
    """LDS-array cycles one ADMM iteration occupies per wave, conflict-free (the planner's
    lds_layout.cpp cost model floor, tests/test_schedule.py): a ds_read_b64 serves its two 32-lane
    halves in 2 cycles, a ds_add_f64 (read-modify-write) its four 16-lane groups in 4 -- so the
    atomics are priced at their real array cost, not as 16 bytes at the read rate -- and each
    64-lane register slot of the vector passes costs 10 (rhs + C store, the D^-1 pass, the
    read-back)."""
    need_n, need_m, need_k = -(-n // 64), -(-m // 64), (n + m) // 64 + 1
    slots = next(3 * b for b in (2, 4, 8) if need_n <= b and need_m <= 2 * b and 3 * b >= need_k)
    return (nfwd + nbwd) * (16 * 2 + atomics_per_step * 4) + 10 * slots


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
    reference's per-step update(l, u) + update(Ax) + warm solve.  Only the oracle calls are timed;
    chasers that terminated (skipped by the engine) are left out of the timed solves and of the
    agreement figures.  Step 0 is the cold solve (set-up data); its agreement with the engine is
    reported separately, and over the solves both sides finish within FAST_ITERS iterations."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    import scipy.sparse as sp
    from mpc_arpo_project_amd.closed_loop import BatchClosedLoop

    S = min(sample, X0.shape[0])
    cl = BatchClosedLoop(prob, X0[:S], device=device, eps_abs=eps, eps_rel=eps)
    rec = []
    for k in range(warmup + steps):
        Ax, l, u = cl.qp.copy_data()
        act = (cl.done == 0).cpu().numpy()
        r = cl.step()
        rec.append((Ax.cpu().numpy(), l.cpu().numpy(), u.cpu().numpy(),
                    r.status.cpu().numpy().copy(), r.iter.cpu().numpy().copy(), act))
    cl.close()
    solvers = []
    for b in range(S):
        A = sp.csc_matrix((rec[0][0][b], prob.A.indices, prob.A.indptr), shape=prob.A.shape)
        s = orc.OracleOSQP()
        s.setup(prob.P, prob.q, A, rec[0][1][b], rec[0][2][b], eps_abs=eps, eps_rel=eps,
                warm_start=True, verbose=False)
        solvers.append(s)
    agree, fast_agree = [], []
    t_cpu, n_timed = 0.0, 0
    for k in range(warmup + steps):
        act = rec[k][5]
        idx = np.flatnonzero(act)
        sv = [solvers[b] for b in idx]
        if k == 0:
            _, st, it = orc.batch_update_solve(sv, None, None, None, threads)
        else:
            t0 = time.perf_counter()
            _, st, it = orc.batch_update_solve(sv, rec[k][0][idx], rec[k][1][idx],
                                               rec[k][2][idx], threads)
            dt = time.perf_counter() - t0
            if k >= warmup:
                t_cpu += dt
                n_timed += len(idx)
        gs, gi = rec[k][3][idx], rec[k][4][idx]
        same = (st == gs) & (it == gi)
        fast = np.maximum(it, gi) <= FAST_ITERS
        agree.append(float(np.mean(st == gs)) if len(idx) else 1.0)
        fast_agree.append(float(np.mean(same[fast])) if fast.any() else 1.0)
    timed = max(steps if warmup >= 1 else steps - 1, 1)
    return dict(value=n_timed / t_cpu, unit="solves/s", cores=threads, kind="port",
                affinity_cpus=len(os.sched_getaffinity(0)), cgroup_cpu_quota=cgroup_cpus(),
                sample=f"{S} chasers x {timed} warm closed-loop steps (update(l,u)+update(Ax)+solve, "
                       f"eps {eps:g}) after {warmup} untimed steps: {n_timed} solves in "
                       f"{t_cpu:.2f} s on {threads} threads",
                status_agreement_with_gpu=float(np.mean(agree)),
                status_agreement_per_step=[round(a, 5) for a in agree],
                cold_step_status_agreement=agree[0],
                cold_step_exact_agreement_within_1000_iters=fast_agree[0],
                warm_exact_agreement_within_1000_iters=float(np.mean(fast_agree[1:])) if
                len(fast_agree) > 1 else None,
                note="free-running: each oracle solver carries its own warm state, so one "
                     "status flip changes its later starting points; see DESIGN.md, Parity")


def load_profile(name, B, nx, split, dv=False, kind="discrete"):
    """A committed PMC-derived figure (profiles/current/<name>.json, <name>_n<nx>[dv].json or, for
    the continuous-time loop, <name>_n<nx>cont.json; written by tools/pmc_traffic.py or
    tools/sq_summary.py on the GPU box) for this workload, with the commit it was measured at."""
    stem = name[:-len(".json")]
    for fn in (name, f"{stem}_n{nx}{'dv' if dv else ''}.json", f"{stem}_n{nx}cont.json"):
        try:
            pj = json.load(open(os.path.join(REPO, "profiles", "current", fn)))
        except Exception:
            continue
        if (pj.get("batch") == B and pj.get("nx") == nx and pj.get("concurrent_shards", 1) == split
                and bool(pj.get("dv", False)) == bool(dv) and pj.get("kind", "discrete") == kind):
            return pj
    return None


def closed_loop_run(prob, X0, B, K, W, S, eps, rank, device, dist=None, track=None,
                    longest_first=False):
    """The timed closed loop: S shards of the B chasers on concurrent HIP streams, one cold solve
    (step 0, timed on its own), W - 1 more untimed warm steps, K timed warm steps bracketed by
    barrier + synchronize.  Per step and chaser it keeps the iterations, status and whether the
    engine solved it (active: not terminated).  track: (nsim, dist_tol, ang_tol) -> per-chaser
    run summaries (enable_tracking)."""
    import torch
    from mpc_arpo_project_amd.closed_loop import BatchClosedLoop, shard_streams

    cut = [B * j // S for j in range(S + 1)]
    cls = []
    sts = shard_streams(device, S) if S > 1 else [None]  # the same streams for every leg
    for j in range(S):
        cls.append(BatchClosedLoop(prob, X0[cut[j]:cut[j + 1]], device=device, eps_abs=eps,
                                   eps_rel=eps, stream=sts[j], id_offset=rank * B + cut[j],
                                   longest_first=longest_first))
        if track:
            cls[-1].enable_tracking(*track)
    torch.cuda.synchronize()
    cold_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(S)]
    cold_it = torch.zeros(B, dtype=torch.int32, device=device)
    cold_act = torch.zeros(B, dtype=torch.bool, device=device)
    torch.cuda.synchronize()
    tc0 = time.perf_counter()
    for j, c in enumerate(cls):
        with torch.cuda.stream(c.qp.stream):
            cold_act[cut[j]:cut[j + 1]].copy_(c.done == 0, non_blocking=True)
        cold_ev[j][0].record(c.qp.stream)
        r = c.qp.solve_async()
        cold_ev[j][1].record(c.qp.stream)
        with torch.cuda.stream(c.qp.stream):
            cold_it[cut[j]:cut[j + 1]].copy_(r.iter, non_blocking=True)
        c.step_after_solve(r)
    torch.cuda.synchronize()
    cold_wall = time.perf_counter() - tc0
    for _ in range(max(W - 1, 0)):
        for c in cls:
            c.step()
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(K)] for _ in range(S)]
    iters = torch.zeros(K, B, dtype=torch.int32, device=device)
    rhou = torch.zeros(K, B, dtype=torch.int32, device=device)
    stat = torch.zeros(K, B, dtype=torch.int32, device=device)
    act = torch.zeros(K, B, dtype=torch.bool, device=device)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        for j, c in enumerate(cls):
            stream = c.qp.stream
            with torch.cuda.stream(stream):
                act[k, cut[j]:cut[j + 1]].copy_(c.done == 0, non_blocking=True)
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
    kt = np.array([[a.elapsed_time(b) for a, b in ev[j]] for j in range(S)]) * 1e-3
    kt_cold = np.array([a.elapsed_time(b) for a, b in cold_ev]) * 1e-3
    return dict(cls=cls, cut=cut, elapsed=elapsed, kt=kt, kt_cold=kt_cold, cold_wall=cold_wall,
                it=iters.cpu().numpy(), ru=rhou.cpu().numpy(), st=stat.cpu().numpy(),
                act=act.cpu().numpy(), cold_it=cold_it.cpu().numpy(),
                cold_act=cold_act.cpu().numpy(), dims=cls[0].qp.dims(),
                sched=cls[0].qp.schedule_info())


def roofline(run, S, K, elapsed):
    """LDS-graded roofline of the solve kernel over the timed region, with the HBM (PMC),
    FP64 and SURVEY streaming-model figures beside it."""
    it, ru, act, cut = run["it"], run["ru"], run["act"], run["cut"]
    dims, sched, kt = run["dims"], run["sched"], run["kt"]
    n, m, nnzA, nnzL = dims["n"], dims["m"], dims["nnzA"], dims["nnzL"]
    b_iter, b_fact, b_io = bytes_model(n, m, nnzA, nnzL)
    lds_iter = lds_bytes_per_iter(sched["fwd_steps"], sched["bwd_steps"], n, m,
                                  sched["atomics_per_step"])
    cyc_iter = lds_cycles_per_iter(sched["fwd_steps"], sched["bwd_steps"], n, m,
                                   sched["atomics_per_step"])
    itm = np.where(act, it, 0).astype(np.float64)
    chk = np.ceil(itm / 25.0)
    # per launch (shard j, step k): LDS bytes, flops, streaming-model bytes of its solved instances
    iters_launch = np.stack([[itm[k, cut[j]:cut[j + 1]].sum() for k in range(K)] for j in range(S)])
    lds_b = iters_launch * lds_iter
    flops = np.stack([[float(np.where(act[k, cut[j]:cut[j + 1]], flops_per_solve(
        itm[k, cut[j]:cut[j + 1]], n, m, nnzA, nnzL, chk[k, cut[j]:cut[j + 1]]), 0).sum())
        for k in range(K)] for j in range(S)])
    per_solve = np.where(act, itm * b_iter + (1 + ru) * b_fact + b_io, 0)
    stream_b = np.stack([per_solve[:, cut[j]:cut[j + 1]].sum(axis=1) for j in range(S)])
    # with S > 1 the shards' launches overlap, so a launch's own duration undercounts; `achieved`
    # = all bytes of the timed region / its wall time (conservative: the gaps between launches
    # count too); the per-launch form (bytes of one launch / its HIP-event duration) beside it
    lds_ach = float(lds_b.sum() / elapsed) / 1e9
    cyc_ach = float(itm.sum() * cyc_iter / elapsed) / 1e9  # LDS-array G cycles / s, chip-wide
    return dict(
        bound="lds", achieved=lds_ach, peak=LDS_PEAK_GBS, unit="GB/s", frac=lds_ach / LDS_PEAK_GBS,
        traffic=None, kernel=kernel_name(sched), kernel_ms_per_launch=float(np.mean(kt) * 1e3),
        concurrent_shards=S, lds_bytes_per_iter=lds_iter,
        admm_iters_timed=float(itm.sum()),
        lds_bytes_per_launch=float(lds_b.mean()),
        achieved_per_launch=float(np.mean(lds_b / kt)) / 1e9,
        recompute="achieved = admm_iters_timed * lds_bytes_per_iter / (ms_per_step * steps / 1e3)",
        why="one QP per wave with the KKT factor and solve vector in LDS: the solve steps are LDS "
            "read/atomic passes; HBM carries only per-solve I/O and check reloads",
        lds_array_cycles={
            "achieved": cyc_ach, "peak": 256 * LDS_CLK_GHZ, "unit": "G LDS-array cycles/s",
            "frac": cyc_ach / (256 * LDS_CLK_GHZ), "cycles_per_iter": cyc_iter,
            "what": "atomic-aware LDS roof: the conflict-free array cycles of the solve steps and "
                    "vector passes (ds_read_b64 2, ds_add_f64 4 per wave-instruction) over one "
                    "cycle per clock per CU; the measured busy share incl. conflicts and the other "
                    "phases is lds_busy"},
        fp64={"achieved": float(flops.sum() / elapsed) / 1e9, "peak": FP64_PEAK_GFLOPS,
              "unit": "GFLOP/s", "frac": float(flops.sum() / elapsed) / 1e9 / FP64_PEAK_GFLOPS},
        survey_streaming_model={
            "model_GBs_if_streamed": float(stream_b.sum() / elapsed) / 1e9,
            "bytes_model": {"per_iter": b_iter, "per_factor": b_fact, "per_solve_io": b_io},
            "note": "a MODEL, not a measurement: SURVEY 8(d)'s bytes if the factor and iterates "
                    "were streamed from HBM every iteration; they stay in LDS / VGPRs, so no HBM "
                    "fraction is claimed from it (the measured HBM figure is `hbm`)"})


def _sources_match(pj):
    """True when the committed profile was measured on a library built from exactly this tree's
    sources (its src_digest, _lib.source_digest); None for profiles that predate the digest"""
    from mpc_arpo_project_amd._lib import source_digest

    return None if "src_digest" not in pj else pj["src_digest"] == source_digest()


def attach_profiles(roof, B, nx, S, K, elapsed, dv=False, kind="discrete"):
    """HBM traffic (PMC FETCH_SIZE + WRITE_SIZE) and LDS busy share (SQ_LDS_IDX_ACTIVE) from the
    committed profile of this workload, when there is one."""
    pj = load_profile("pmc_traffic.json", B, nx, S, dv, kind)
    if pj and pj.get("hbm_bytes_per_launch"):
        t = pj["hbm_bytes_per_launch"]
        ach = t * S * K / elapsed / 1e9
        roof["traffic"] = t
        roof["hbm"] = {"achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": ach / HBM_PEAK_GBS, "bytes_per_launch": t,
                       "bytes_per_solve": pj.get("hbm_bytes_per_solve"),
                       "measured_at": pj.get("commit"),
                       "sources_match": _sources_match(pj),
                       "what": "PMC FETCH_SIZE + WRITE_SIZE (L2 <-> fabric, calibrated; "
                               "tools/pmc_run.sh)"}
    sq = load_profile("sq_summary.json", B, nx, S, dv, kind)
    if sq and sq.get("lds_array_busy_fraction_if_per_cu") is not None:
        roof["lds_busy"] = {"frac": sq["lds_array_busy_fraction_if_per_cu"],
                            "bank_conflict_share": sq.get("lds_conflict_share"),
                            "measured_at": sq.get("commit"),
                            "sources_match": _sources_match(sq),
                            "what": "SQ_LDS_IDX_ACTIVE / CU cycles of the solve kernel (all LDS-"
                                    "array cycles, atomics at their real cost; tools/pmc_sq.sh)"}


def bench_discrete(args, rank, world, device, dist):
    from mpc_arpo_project_amd import launch as _launch, qp_model, scenarios

    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=args.nx, isDeltaV=args.dv)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    B, K, S = args.batch, args.steps, max(1, min(args.split, args.batch))
    X0 = initial_states(world * B, rank, B, args.seed)
    run = closed_loop_run(prob, X0, B, K, args.warmup, S, args.eps, rank, device, dist,
                          longest_first=args.order == "iters",
                          track=(int(sim.T_final / sim.time_stp), *sim.suc_cond))
    cls = run["cls"]
    elapsed = run["elapsed"]
    # after the timed region: the per-chaser run summaries (first MPC input, last
    # status, ADMM iterations, i_term, success, final error, fallback steps) of every rank, one
    # all-gather (RCCL over xGMI)
    import torch

    summ = _launch.gather_rows(torch.cat([c.summary() for c in cls]), world * B, rank, world, dist)
    solved = float(run["act"].sum())
    if dist:
        t = torch.tensor([elapsed, solved], dtype=torch.float64, device=device)
        tt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(tt, t)
        elapsed = max(float(x[0]) for x in tt)
        solved = sum(float(x[1]) for x in tt)
    roof = roofline(run, S, K, run["elapsed"])
    attach_profiles(roof, B, args.nx, S, K, run["elapsed"], args.dv)
    if rank != 0:
        for c in cls:
            c.close()
        return None
    it, st, act = run["it"], run["st"], run["act"]
    uniq, cnt = np.unique(st[act], return_counts=True)
    Sn = summ.cpu().numpy()
    ci = run["cold_it"][run["cold_act"]]
    dims = run["dims"]
    metric = METRIC if (args.nx, args.dv) == (20, False) else (
        f"MPC-QP solves/sec @ N={args.nx}{', impulsive delta-v' if args.dv else ''}, CW, "
        f"batch={B}; ADMM iters to {args.eps:g}")
    out = {
        "metric": metric,
        "value": solved / elapsed,
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
                        f"settings with eps_abs=eps_rel={args.eps:g}; chasers start at rest at "
                        f"SURVEY 8(d)'s sampled positions (velocities 0 as the reference's x0, no "
                        f"disturbance estimate: noise=None; the cold parity fixtures use the full "
                        f"generator)",
            "batch_per_gpu": B,
            "global_batch": world * B,
            "N": args.nx,
            "parallelism": f"shard{world}" if world > 1 else "single",
            "streams_per_gpu": S,
        },
        "solves": {"counted": int(solved), "offered": int(world * B * K),
                   "what": "value counts the solves the engine ran; terminated chasers are "
                           "skipped (reference src/trajectorySimulate.py:288-293)"},
        "roofline": roof,
        "cold": {"value": float(run["cold_act"].sum()) * world / run["cold_wall"],
                 "unit": "solves/s", "wall_ms": run["cold_wall"] * 1e3,
                 "kernel_ms_per_launch": float(run["kt_cold"].mean() * 1e3),
                 "admm_iters_mean": float(ci.mean()) if len(ci) else None,
                 "what": "step 0: every chaser solved once from its set-up data, no warm start"},
        "admm_iters": {"mean": float(it[act].mean()), "median": float(np.median(it[act])),
                       "p90": float(np.percentile(it[act], 90)), "max": int(it[act].max())},
        "status_counts": {str(int(a)): int(c) for a, c in zip(uniq, cnt)},
        "schedule": run["sched"],
        "summary_gather": {"rows": int(Sn.shape[0]), "fields": list(cls[0].SUMMARY_FIELDS),
                           "bytes": int(Sn.nbytes),
                           "mean_admm_iters_per_chaser": float(Sn[:, 3].mean())},
    }
    for c in cls:
        c.close()
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
    return out


def kernel_name(sched):
    """the solve kernel a handle launches: one wave per instance, or two"""
    return "qp_pair_kernel" if sched.get("waves_per_instance", 1) == 2 else "qp_batch_kernel"


def lds_roof(iters_total, lds_iter, seconds, kernel_ms=None, fp64=None, kernel="qp_batch_kernel",
             cyc_iter=None):
    """LDS-graded roofline of a leg: the LDS bytes its solve launches moved (ADMM iterations x
    lds_bytes_per_iter) over the leg's timed wall time (and the atomic-aware array-cycle roof)."""
    ach = iters_total * lds_iter / seconds / 1e9
    out = {"bound": "lds", "achieved": ach, "peak": LDS_PEAK_GBS, "unit": "GB/s",
           "frac": ach / LDS_PEAK_GBS, "traffic": None, "kernel": kernel,
           "lds_bytes_per_iter": lds_iter, "admm_iters_timed": float(iters_total)}
    if cyc_iter is not None:
        ca = iters_total * cyc_iter / seconds / 1e9
        out["lds_array_cycles"] = {"achieved": ca, "peak": 256 * LDS_CLK_GHZ,
                                   "unit": "G LDS-array cycles/s", "frac": ca / (256 * LDS_CLK_GHZ),
                                   "cycles_per_iter": cyc_iter}
    if kernel_ms is not None:
        out["kernel_ms_per_launch"] = kernel_ms
    if fp64 is not None:
        out["fp64"] = fp64
    return out


def bench_leg(args, rank, device, nx, dv, batch=None, split=None, label=None):
    """A discrete closed-loop leg in the same run, at the headline's window (args.steps timed
    after args.warmup): N = 40 impulsive delta-v (BASELINE config 3, reference
    src/trajectorySimulate.py:110-111) and N = 40 continuous acceleration (the horizon every
    reference script runs: test/traj_eval_radial.py:57), B = 65,536 chasers each."""
    from mpc_arpo_project_amd import qp_model, scenarios

    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=nx, isDeltaV=dv)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    B = batch or args.batch
    S = max(1, min(split or args.split, B))
    K = args.leg_steps or args.steps
    W = args.leg_warmup if args.leg_warmup is not None else args.warmup
    X0 = initial_states(B, 0, B, args.seed)
    run = closed_loop_run(prob, X0, B, K, W, S, args.eps, rank, device, None, track=None,
                          longest_first=args.order == "iters")
    it, act = run["it"], run["act"]
    roof = roofline(run, S, K, run["elapsed"])
    attach_profiles(roof, B, nx, S, K, run["elapsed"], dv)
    for c in run["cls"]:
        c.close()
    model = "impulsive delta-v" if dv else "continuous acceleration"
    return {"metric": f"MPC-QP solves/sec @ N={nx}, {model}, CW, batch={B}; ADMM iters to "
                      f"{args.eps:g}" + (f" ({label})" if label else ""),
            "initial_states": "at rest at SURVEY 8(d)'s sampled positions (noise=None)",
            "value": float(act.sum()) / run["elapsed"], "unit": "solves/s", "steps": K,
            "warmup": W, "ms_per_step": run["elapsed"] / K * 1e3,
            "config": {"workload": f"warm closed-loop MPC-QP solves, radial CW scenario, N=Nx={nx}, "
                                   f"Nc=Nb=5, {model} (n={run['dims']['n']}, "
                                   f"m={run['dims']['m']})", "batch_per_gpu": B,
                       "streams_per_gpu": S},
            "roofline": {k: roof[k] for k in ("bound", "achieved", "peak", "unit", "frac",
                                              "traffic", "kernel", "kernel_ms_per_launch",
                                              "lds_bytes_per_iter", "admm_iters_timed", "fp64",
                                              "lds_array_cycles", "hbm", "lds_busy")
                         if k in roof},
            "admm_iters": {"mean": float(it[act].mean()), "median": float(np.median(it[act])),
                           "p90": float(np.percentile(it[act], 90)), "max": int(it[act].max())},
            "schedule": run["sched"]}


def bench_continuous(args, rank, world, device, dist):
    """BASELINE config 4: trajectorySimulateC's loop (reference src/trajectorySimulateC.py:325-405)
    for B chasers -- at every 0.5 s sample instant the warm-started offset-free MPC solve
    (isReject=True, the disturbance-augmented model), then 500 RK45 sub-steps of the nonlinear
    plant at T_cont = 1 ms with the control held, then the UKF update and the QP rebuild
    (reference test/traj_eval_radialC.py: Nx = 40, noise (0.0012, 0.0012) held 50 samples).
    A step is one sample period; value = QP solves per second over the timed periods, with the
    per-period split of the solve, plant + UKF + configure time (HIP events; shard 0's stream when
    the loop runs as --cont-split shards on concurrent HIP streams, ShardedClosedLoopC)."""
    import torch
    from mpc_arpo_project_amd import qp_model, scenarios
    from mpc_arpo_project_amd.closed_loop import BatchClosedLoopC, ShardedClosedLoopC
    from mpc_arpo_project_amd.mpcsim import Noise

    nx = args.nx if args.nx != 20 else 40
    noise = Noise((0.0012, 0.0012), 50)
    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=nx, isDeltaV=args.dv, noise=noise,
                                                    T_final=300, T_cont=0.001)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    B, K, W = args.batch, args.steps, args.warmup
    X0 = initial_states(world * B, rank, B, args.seed)
    S = max(1, min(args.cont_split, B))
    kw = dict(T_cont=0.001, T_final=300, mean_motion=sim.mean_mtn, isDeltaV=args.dv, device=device,
              noise=noise, id_offset=rank * B, eps_abs=args.eps, eps_rel=args.eps,
              longest_first=args.order == "iters")
    cl = ShardedClosedLoopC(prob, X0, shards=S, **kw) if S > 1 else BatchClosedLoopC(prob, X0, **kw)
    parts = cl.parts if S > 1 else [cl]
    cut = cl.cut if S > 1 else [0, B]
    for _ in range(W):
        cl.period()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    iters = torch.zeros(K, B, dtype=torch.int32, device=device)
    act = torch.zeros(K, B, dtype=torch.bool, device=device)
    stream = parts[0].qp.stream
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        for j, c in enumerate(parts):  # each shard's bookkeeping on its own stream
            with torch.cuda.stream(c.qp.stream):
                act[k, cut[j]:cut[j + 1]].copy_(c.done == 0, non_blocking=True)
        ev[k][0].record(stream)
        rs = []
        for j, c in enumerate(parts):
            rs.append(c.period(on_solved=ev[k][1].record if j == 0 else None))
            if j == 0:
                ev[k][2].record(stream)
        for j, c in enumerate(parts):
            with torch.cuda.stream(c.qp.stream):
                iters[k, cut[j]:cut[j + 1]].copy_(rs[j].iter, non_blocking=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    a = act.cpu().numpy()
    it = iters.cpu().numpy()
    solved = float(a.sum())
    if dist:
        t = torch.tensor([elapsed, solved], dtype=torch.float64, device=device)
        tt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(tt, t)
        elapsed = max(float(x[0]) for x in tt)
        solved = sum(float(x[1]) for x in tt)
    sched = cl.qp.schedule_info()
    dims = cl.qp.dims()
    nsub = cl.schedule[W][1] if W < len(cl.schedule) else None
    cl.close()
    if rank != 0:
        return None
    t_solve = np.array([e[0].elapsed_time(e[1]) for e in ev])
    t_rest = np.array([e[1].elapsed_time(e[2]) for e in ev])
    lds_iter = lds_bytes_per_iter(sched["fwd_steps"], sched["bwd_steps"], dims["n"], dims["m"],
                                  sched["atomics_per_step"])
    it_timed = float(np.where(a, it, 0).sum())
    # graded over the whole timed periods (plant + UKF + configure included); the solve launches
    # alone beside it (their HIP-event time)
    roof = lds_roof(it_timed, lds_iter, elapsed, kernel_ms=float(t_solve.mean()),
                    kernel=kernel_name(sched),
                    cyc_iter=lds_cycles_per_iter(sched["fwd_steps"], sched["bwd_steps"], dims["n"],
                                                 dims["m"], sched["atomics_per_step"]))
    roof["concurrent_shards"] = S
    if S == 1:  # with shards the solve launches overlap: their own time is not the loop's share
        roof["frac_over_solve_launches"] = it_timed * lds_iter / (t_solve.sum() * 1e-3) / 1e9 / LDS_PEAK_GBS
    attach_profiles(roof, B, nx, S, K, elapsed, args.dv, kind="continuous")
    return {
        "metric": f"MPC-QP solves/sec @ N={nx} offset-free MPC in the continuous-time nonlinear "
                  f"loop (trajectorySimulateC), batch={B}; ADMM iters to {args.eps:g}",
        "value": solved / elapsed, "unit": "solves/s", "n_gpus": world, "steps": K,
        "warmup": W, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded chaser states in the LOS cone; radial continuous-time scenario "
                "of reference test/traj_eval_radialC.py, device noise stream)",
        "config": {"workload": f"one sample period per step: warm MPC-QP solve (N=Nx={nx}, n="
                               f"{dims['n']}, m={dims['m']}, isReject=True) + {nsub} RK45 plant "
                               f"sub-steps at 1 ms (control held) + UKF + configure",
                   "batch_per_gpu": B, "global_batch": world * B, "N": nx,
                   "parallelism": f"shard{world}" if world > 1 else "single",
                   "streams_per_gpu": S},
        "roofline": roof,
        "period_split_ms": {"solve": float(t_solve.mean()),
                            "plant_ukf_configure": float(t_rest.mean()),
                            "of": "shard 0" if S > 1 else "the loop"},
        "admm_iters": {"mean": float(it[a].mean()) if a.any() else None,
                       "p90": float(np.percentile(it[a], 90)) if a.any() else None},
        "schedule": sched,
    }


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
    ap.add_argument("--cont-split", type=int, default=3,
                    help="concurrent HIP-stream shards of the continuous-time loop (config 4; "
                         "measured 183.5k / 192.2k / 194.1k solves/s with 1 / 2 / 3)")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the N=40 legs (config 3 delta-v, N=40 continuous acceleration, "
                         "config 4 continuous-time loop) of the default run")
    ap.add_argument("--leg-steps", type=int, default=0,
                    help="timed steps of the N=40 discrete legs (default: --steps)")
    ap.add_argument("--leg-warmup", type=int, default=None,
                    help="untimed steps of the N=40 discrete legs (default: --warmup)")
    ap.add_argument("--cont-steps", type=int, default=5,
                    help="timed sample periods of the config-4 leg of the default run")
    ap.add_argument("--continuous", action="store_true",
                    help="BASELINE config 4: the continuous-time nonlinear loop (default N=40)")
    ap.add_argument("--order", choices=("iters", "none"), default="none",
                    help="solve order of each launch: longest-first by the chaser's last ADMM "
                         "iterations (mpcqp_set_order) or instance order")
    ap.add_argument("--split", type=int, default=2,
                    help="chaser shards per GPU on concurrent HIP streams (fills one shard's solve "
                         "tail with the other shard's work; 2 measured best, 4 no better than 1)")
    args = ap.parse_args(argv[1:])
    if args.gpus > 1 and not launch.launched():
        # one process per GPU: start torch.distributed.run as a child (nothing has touched the
        # GPU in this process) and exit with its status
        return launch.relaunch(args.gpus, argv)

    rank, world, local, device, dist = launch.init("nccl")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but {world} ranks were launched")
    if args.continuous:
        out = bench_continuous(args, rank, world, device, dist)
    else:
        out = bench_discrete(args, rank, world, device, dist)
        default_cfg = (args.nx, args.dv) == (20, False)
        if out is not None and world == 1 and default_cfg and not args.no_legs:
            for key, nx, dv in (("config3", 40, True), ("n40_accel", 40, False)):
                try:
                    out[key] = bench_leg(args, rank, device, nx, dv)
                except Exception as e:  # report, never fake
                    out[key] = {"error": repr(e)}
            try:  # BASELINE config 2: B = 1,024 at N = 20, one launch (latency-bound: one grid)
                out["config2"] = bench_leg(args, rank, device, 20, False, batch=1024, split=1,
                                           label="BASELINE config 2")
            except Exception as e:  # report, never fake
                out["config2"] = {"error": repr(e)}
            try:
                ca = argparse.Namespace(**vars(args))
                ca.nx, ca.dv, ca.steps, ca.warmup = 40, False, args.cont_steps, 1
                out["config4"] = bench_continuous(ca, rank, world, device, dist)
            except Exception as e:  # report, never fake
                out["config4"] = {"error": repr(e)}
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
