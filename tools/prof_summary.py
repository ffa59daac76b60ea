"""Summarise a rocprofv3 kernel trace of bench.py: the solve kernel's per-launch duration over the
TIMED launches only (the first `--warmup` launches are bench.py's untimed warm-up steps), so it can
be compared with the HIP-event `kernel_ms_per_launch` that bench.py reports.

    python tools/prof_summary.py <run_kernel_trace.csv> <bench.json> [--warmup 3] > summary.json
"""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--kernel", default=None, help="default: the kernel the bench's roofline names")
    a = ap.parse_args()
    bench = json.loads(open(a.bench).read().strip().splitlines()[-1])
    # the untimed warm-up steps launch the solve kernel once per concurrent shard
    warm = bench["warmup"] * bench["roofline"].get("concurrent_shards", 1) if a.warmup is None else a.warmup
    kname = a.kernel or bench["roofline"].get("kernel", "qp_batch_kernel")
    rows = [r for r in csv.DictReader(open(a.trace)) if kname in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]) * 1e-6
    timed = dur[warm:]
    r0 = rows[0]
    out = {
        "kernel": r0["Kernel_Name"],
        "launches_total": len(rows),
        "launches_timed": int(timed.size),
        "rocprof_ms_per_launch_timed": float(timed.mean()),
        "rocprof_ms_min": float(timed.min()),
        "rocprof_ms_max": float(timed.max()),
        "bench_hip_event_ms_per_launch": bench["roofline"]["kernel_ms_per_launch"],
        "agreement": float(timed.mean() / bench["roofline"]["kernel_ms_per_launch"]),
        "vgpr": int(r0["VGPR_Count"]), "agpr": int(r0["Accum_VGPR_Count"]),
        # rocprofv3 derives VGPR_Count from the code object's granulated register count with the
        # pre-gfx90a granule of 4; gfx950's unified VGPR + AGPR file is allocated in granules of 8
        # (MI355X_MICROARCH.md, Register files), so the registers a wave holds are twice the
        # reported count, AGPRs included (Accum_VGPR_Count reads 0): 208 -> 416 >= 256 + 154
        "unified_regs_allocated": 2 * int(r0["VGPR_Count"]),
        "waves_per_simd_by_regs": min(8, 512 // (2 * int(r0["VGPR_Count"]))),
        "sgpr": int(r0["SGPR_Count"]), "lds_bytes": int(r0["LDS_Block_Size"]),
        "scratch": int(r0["Scratch_Size"]), "workgroup": int(r0["Workgroup_Size_X"]),
        "grid": int(r0["Grid_Size_X"]),
    }
    # per HIP stream (concurrent shards): the continuous-time bench times shard 0's solve only
    # (period_split_ms), so its figure is compared with the launches on shard 0's stream -- the
    # stream of the first launch (shard 0 is enqueued first in every period)
    streams = {}
    for r, d in zip(rows[warm:], timed):
        streams.setdefault(r.get("Stream_Id", "0"), []).append(float(d))
    out["per_stream_ms_per_launch"] = {k: float(np.mean(v)) for k, v in streams.items()}
    if "period_split_ms" in bench:
        s0 = rows[0].get("Stream_Id", "0")
        out["agreement_all_streams"] = out["agreement"]
        out["agreement"] = float(np.mean(streams[s0]) / bench["roofline"]["kernel_ms_per_launch"])
        out["agreement_of"] = "shard 0's stream (the bench times shard 0's solve)"
    # the engine's own figure (hipFuncGetAttributes of the selected kernel, bench schedule); rocprof
    # reports the allocation in whole granules of 8 registers
    kr = bench.get("schedule", {}).get("kernel_regs")
    out["schedule_kernel_regs"] = kr
    out["regs_match"] = None if kr is None else out["unified_regs_allocated"] == -(-kr // 8) * 8
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
