"""HBM traffic per launch of the QP kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one TCC pass), each
counter is calibrated against a known byte count of the kernel's own access width (tools/pmc_calib,
8 bytes per lane), and the bench's untimed warm-up launches are dropped.

    python tools/pmc_traffic.py --fetch DIR --write DIR --calib-fetch DIR --calib-write DIR \
        --bench bench.json --out profiles/pmc_traffic.json
"""
import argparse
import csv
import glob
import json
import os

import numpy as np


def per_dispatch(d, kernel, counter):
    """{dispatch_id: value} of `counter` summed over its instances, for dispatches of `kernel`."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--bench", required=True, help="bench.py JSON line of the PMC runs' workload")
    ap.add_argument("--calib-bytes", type=float, default=float(1 << 30))
    ap.add_argument("--kernel", default=None, help="default: the kernel the bench roofline names")
    ap.add_argument("--dv", action="store_true", help="the impulsive delta-v model (bench --dv)")
    ap.add_argument("--kind", default="discrete", help="discrete (closed-loop steps) or continuous "
                    "(bench.py --continuous: one solve launch per sample period)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    bench = json.loads(open(a.bench).read().strip().splitlines()[-1])
    a.kernel = a.kernel or bench["roofline"].get("kernel", "qp_batch_kernel")
    S = bench["roofline"].get("concurrent_shards", 1)  # solve launches per step (one per shard)
    warm = bench["warmup"] * S

    cf = np.array(per_dispatch(a.calib_fetch, "calib_read8", "FETCH_SIZE"))
    cw = np.array(per_dispatch(a.calib_write, "calib_write8", "WRITE_SIZE"))
    # counters report kilobytes; the factor maps a reported unit to true bytes for 8 B/lane access
    f_fetch = a.calib_bytes / float(np.median(cf))
    f_write = a.calib_bytes / float(np.median(cw))

    fe = np.array(per_dispatch(a.fetch, a.kernel, "FETCH_SIZE"))[warm:]
    wr = np.array(per_dispatch(a.write, a.kernel, "WRITE_SIZE"))[warm:]
    read_b = float(fe.mean()) * f_fetch
    write_b = float(wr.mean()) * f_write
    rl = bench["roofline"]
    if S == 1:
        alg = rl["achieved"] * 1e9 * rl["kernel_ms_per_launch"] * 1e-3
    else:  # achieved is over the wall time of the timed region; one step = S launches
        alg = rl["achieved"] * 1e9 * bench["ms_per_step"] * 1e-3 / S
    per_launch = bench["config"]["batch_per_gpu"] // S
    out = {
        "batch": bench["config"]["batch_per_gpu"],
        "nx": bench["config"]["N"],
        "launches": int(min(fe.size, wr.size)),
        "fetch_size_raw_mean": float(fe.mean()),
        "write_size_raw_mean": float(wr.mean()),
        "calib": {"fetch_bytes_per_unit": f_fetch, "write_bytes_per_unit": f_write,
                  "calib_bytes": a.calib_bytes, "access": "8 B/lane coalesced (tools/pmc_calib.hip)"},
        "hbm_read_bytes_per_launch": read_b,
        "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "solves_per_launch": per_launch,
        "concurrent_shards": S,
        "hbm_bytes_per_solve": (read_b + write_b) / per_launch,
        "kind": a.kind,
        "dv": bool(a.dv),
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
