"""Post-process tools/profile_r5.sh output (here, after gpurun merged gpurun_out/<tag>/) into the
committed profile files: profiles/current/ (what bench.py attaches: PMC HBM traffic per launch and
the SQ LDS-busy share, each with the workload it belongs to and the commit it was measured at) and
profiles/<round>/final/ (kernel-trace summaries against the bench's HIP-event timings, the PMC and
SQ summaries, the bench lines of the profiled runs).

    python tools/profile_post.py gpurun_out/<tag> profiles/r05/final [--commit SHA]
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(REPO, "tools")
sys.path.insert(0, REPO)
from mpc_arpo_project_amd._lib import source_digest  # noqa: E402

# the sources of the library that was profiled: this tree's (run profile_post on the tree that was
# pushed to the GPU box, before any source edit)
SRC_DIGEST = source_digest()


def run(args):
    return subprocess.check_output([sys.executable] + args, cwd=REPO).decode()


def trace_csv(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    return f[0] if f else None


def meta(bench, kind, dv, commit):
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    return {"batch": b["config"]["batch_per_gpu"], "nx": b["config"]["N"],
            "concurrent_shards": b["roofline"].get("concurrent_shards", 1), "dv": dv, "kind": kind,
            "commit": commit, "src_digest": SRC_DIGEST}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--commit", default=None)
    a = ap.parse_args()
    commit = a.commit or subprocess.check_output(["git", "rev-parse", "--short", "HEAD"],
                                                 cwd=REPO).decode().strip()
    cur = os.path.join(REPO, "profiles", "current")
    os.makedirs(a.dst, exist_ok=True)
    # kernel traces vs HIP events
    for name, tdir, bench in (("", "trace", "bench.json"), ("_n40dv", "trace40", "bench_n40dv.json"),
                              ("_continuous", "trace_cont", "bench_cont.json")):
        t, bj = trace_csv(os.path.join(a.src, tdir)), os.path.join(a.src, bench)
        if not t or not os.path.exists(bj):
            continue
        # the untimed warm-up launches: warmup x concurrent shards (prof_summary's default)
        out = json.loads(run([os.path.join(TOOLS, "prof_summary.py"), t, bj]))
        out.update(commit=commit, src_digest=SRC_DIGEST)
        json.dump(out, open(os.path.join(a.dst, f"prof_summary{name}.json"), "w"), indent=1)
        shutil.copy(bj, os.path.join(a.dst, f"bench{name}.json"))
        st = glob.glob(os.path.join(a.src, tdir, "**", "*kernel_stats.csv"), recursive=True)
        if st:
            shutil.copy(st[0], os.path.join(a.dst, f"kernel_stats{name}.csv"))
    # PMC HBM traffic per launch
    cf, cw = os.path.join(a.src, "calib_fetch"), os.path.join(a.src, "calib_write")
    for n, suffix, kind, dv, extra in (("n20", "", "discrete", False, []),
                                       ("n40dv", "_n40dv", "discrete", True, ["--dv"]),
                                       ("n40", "_n40", "discrete", False, []),
                                       ("cont", "_n40cont", "continuous", False, ["--kind", "continuous"]),
                                       ("c2", "_n20", "discrete", False, [])):  # config 2 (B = 1,024)
        fe, wr = os.path.join(a.src, f"fetch_{n}"), os.path.join(a.src, f"write_{n}")
        bj = os.path.join(a.src, f"bench_fetch_{n}.json")
        if not (os.path.isdir(fe) and os.path.isdir(wr) and os.path.isdir(cf)):
            continue
        outp = os.path.join(a.dst, f"pmc_traffic{suffix}.json")
        run([os.path.join(TOOLS, "pmc_traffic.py"), "--fetch", fe, "--write", wr, "--calib-fetch", cf,
             "--calib-write", cw, "--bench", bj, "--out", outp] + extra)
        pj = json.load(open(outp))
        pj.update(meta(bj, kind, dv, commit))
        json.dump(pj, open(outp, "w"), indent=1)
        shutil.copy(outp, os.path.join(cur, f"pmc_traffic{suffix}.json"))
        shutil.copy(bj, os.path.join(a.dst, f"bench_pmc_{n}.json"))
    # SQ LDS counters
    for n, suffix, kname, dv in (("sq20", "", "qp_batch_kernel", False),
                                 ("sq40", "_n40dv", "qp_pair_kernel", True)):
        d, bj = os.path.join(a.src, n), os.path.join(a.src, f"{n}.json")
        if not os.path.isdir(d):
            continue
        sj = json.loads(run([os.path.join(TOOLS, "sq_summary.py"), "--kernel", kname, d]))
        sj.update(meta(bj, "discrete", dv, commit))
        outp = os.path.join(a.dst, f"sq_summary{suffix}.json")
        json.dump(sj, open(outp, "w"), indent=1)
        shutil.copy(outp, os.path.join(cur, f"sq_summary{suffix}.json"))
    print("\n".join(sorted(os.listdir(a.dst))))


if __name__ == "__main__":
    main()
