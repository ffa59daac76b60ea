"""Mean SQ / GRBM counter values per launch of the solve kernel from rocprofv3 --pmc passes, with
the derived LDS utilisation (MI355X_MICROARCH.md: SQ_LDS_IDX_ACTIVE = LDS-array cycles,
SQ_LDS_BANK_CONFLICT = their conflict part; SQ_* wave counters in quad-cycles; GRBM_GUI_ACTIVE
summed over the 8 XCDs).

    python tools/sq_summary.py [--kernel NAME] DIR [DIR ...] > summary.json

--kernel: substring of the kernel name (default qp_batch_kernel; "qp_batch_kernel<2, 4" keeps the
N = 20 launches when a run also holds the config-3 leg's N = 40 ones)
"""
import csv
import glob
import json
import os
import sys


def main():
    vals = {}
    args = sys.argv[1:]
    kernel = "qp_batch_kernel"
    if args and args[0] == "--kernel":
        kernel, args = args[1], args[2:]
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = {}
            for r in csv.DictReader(open(f)):
                if kernel not in r["Kernel_Name"]:
                    continue
                key = (r["Counter_Name"], int(r["Dispatch_Id"]))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            for (c, _), v in per.items():
                vals.setdefault(c, []).append(v)
    mean = {c: sum(v) / len(v) for c, v in sorted(vals.items())}
    out = {"counters_mean_per_launch": mean, "launches": {c: len(v) for c, v in vals.items()}}
    if "SQ_LDS_IDX_ACTIVE" in mean and "SQ_LDS_BANK_CONFLICT" in mean:
        out["lds_conflict_share"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"]
    if "GRBM_GUI_ACTIVE" in mean and "SQ_LDS_IDX_ACTIVE" in mean:
        # LDS-array busy fraction: LDS cycles per CU over the kernel's active cycles per XCD
        cu_cycles = mean["GRBM_GUI_ACTIVE"] / 8 * 256
        out["lds_array_busy_fraction_if_per_cu"] = mean["SQ_LDS_IDX_ACTIVE"] / cu_cycles
    if "SQ_WAIT_INST_LDS" in mean and "SQ_WAVE_CYCLES" in mean:
        out["wave_cycles_waiting_on_lds_issue"] = mean["SQ_WAIT_INST_LDS"] / mean["SQ_WAVE_CYCLES"]
    if "SQ_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
        out["sq_busy_over_gui_active"] = mean["SQ_BUSY_CYCLES"] / mean["GRBM_GUI_ACTIVE"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
