"""Per-phase cycle breakdown of the QP kernel on the bench workload (diagnostic build).

    python tools/phase_timing.py build            # here: hipcc -DMPCQP_TIMING -> tools/libmpcqp_timing.so
    python tools/phase_timing.py run [B] [steps] [warmup] [nx] [dv]  # GPU box: warm closed loop, prints cycles per phase

The timing build stamps s_memtime around scaling, factorization, forward / backward solves, the
vector work of an ADMM iteration, and the checks (engine.hip, MPCQP_TIMING).  Cycles are s_memtime
ticks (shader clock) summed over all instances of the timed steps.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("MPCQP_TIMING_LIB") or os.path.join(REPO, "tools", "libmpcqp_timing.so")
SLOTS = ["scale", "factor", "fwd", "bwd", "vec", "check", "tail", "iters", "nfact", "resid", "term", "nchk", "adapt",
         "scale_finish", "vec_rhs", "vec_diag", "vec_update", "rs_stage", "rs_matvecs", "chk_on", "chk_off", "rs_norms", "tm_norms", "tm_pinf", "tm_dinf",
         "sc_norms", "sc_factors", "sc_rescale", "sc_cost", "sc_cost_seq_count"]


def build(extra=()):
    csrc = os.path.join(REPO, "mpc_arpo_project_amd", "csrc")
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
           "-DMPCQP_TIMING", *extra, os.path.join(csrc, "engine.hip"),
           os.path.join(csrc, "closed_loop.hip"),
           os.path.join(csrc, "estimation.hip"), os.path.join(csrc, "host_abi.cpp"),
           os.path.join(csrc, "symbolic.cpp"), os.path.join(csrc, "lds_layout.cpp"),
           os.path.join(csrc, "emulate.cpp"), "-o", LIB]
    subprocess.check_call(cmd)


def run(B=65536, steps=5, warmup=3, nx=20, dv=0):
    os.environ["MPCQP_DIAGNOSTICS"] = "1"  # MPCQP_LIBRARY is honoured only with it (_lib.py)
    os.environ["MPCQP_LIBRARY"] = LIB
    sys.path.insert(0, REPO)
    import ctypes as C

    import torch
    from mpc_arpo_project_amd import _lib, qp_model, scenarios
    from mpc_arpo_project_amd.closed_loop import BatchClosedLoop

    L = _lib.lib()
    L.mpcqp_debug_timing.argtypes = [C.c_void_p, C.c_void_p]
    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=nx, isDeltaV=bool(dv))
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    X = scenarios.sample_estimates(B, seed=20250328)[:, :4].copy()
    X[:, 2:4] = 0.0
    cl = BatchClosedLoop(prob, X, device=torch.device("cuda", 0), eps_abs=1e-4, eps_rel=1e-4)
    for _ in range(warmup):
        cl.step()
    buf = torch.zeros(len(SLOTS), dtype=torch.int64, device="cuda")
    L.mpcqp_debug_timing(cl.qp._h, C.c_void_p(buf.data_ptr()))
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kt = 0.0
    for _ in range(steps):
        ev0.record(cl.qp.stream)
        r = cl.qp.solve_async()
        ev1.record(cl.qp.stream)
        cl.step_after_solve(r)
        torch.cuda.synchronize()
        kt += ev0.elapsed_time(ev1)
    t = dict(zip(SLOTS, buf.cpu().tolist()))
    n_inst = B * steps
    iters = t["iters"]
    sched = cl.qp.schedule_info()
    out = {"B": B, "steps": steps, "kernel_ms_per_launch": kt / steps,
           "iters_per_solve": iters / n_inst, "factorizations_per_solve": t["nfact"] / n_inst,
           "cycles_per_solve": {k: t[k] / n_inst for k in SLOTS[:7]},
           "cycles_per_iter": {k: t[k] / iters for k in ("fwd", "bwd", "vec", "check", "vec_rhs", "vec_diag",
                                                         "vec_update")},
           "cycles_per_factorization": t["factor"] / max(t["nfact"], 1),
           "cycles_per_check": {"resid": t["resid"] / max(t["nchk"], 1),
                                "term": t["term"] / max(t["nchk"], 1),
                                "adapt": t["adapt"] / max(t["nchk"], 1),
                                "check_total": t["check"] / max(t["nchk"], 1),
                                **{k: t[k] / max(t["nchk"], 1) for k in SLOTS if k.startswith(("rs_", "tm_"))}},
           # the check slot on the iterations that compute residuals (per such iteration) and on the
           # others (per iteration): the second is the branch + the stamps' own cost
           "check_slot_split": {"per_check_iteration": t["chk_on"] / max(t["nchk"], 1),
                                "per_other_iteration": t["chk_off"] / max(iters - t["nchk"], 1)},
           "scale_finish_per_solve": t["scale_finish"] / n_inst,
           # the Ruiz passes' parts, per pass (scaling passes per solve = settings.scaling, 10)
           "ruiz_cycles_per_pass": {k: t[k] / (10 * n_inst) for k in ("sc_norms", "sc_factors",
                                                                   "sc_rescale", "sc_cost")},
           "ruiz_mean_sequential_share": t["sc_cost_seq_count"] / (10 * n_inst),
           "cycles_per_solve_step": {"fwd": t["fwd"] / iters / sched["fwd_steps"],
                                     "bwd": t["bwd"] / iters / sched["bwd_steps"]},
           "cycles_per_factor_step": t["factor"] / max(t["nfact"], 1) / sched["fac_steps"],
           "schedule": sched}
    tot = sum(t[k] for k in SLOTS[:7])
    out["share"] = {k: t[k] / tot for k in SLOTS[:7]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        args = [int(a) for a in sys.argv[2:]]
        run(*args)
