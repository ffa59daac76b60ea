"""Sum the counter passes of tools/pmc_study.sh over the solve kernel's dispatches and print the
derived ratios (per-pass dispatch sets differ only by timing)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

O = sys.argv[1]
tot = defaultdict(float)
n = defaultdict(int)
for f in sorted(glob.glob(os.path.join(O, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        if "qp_batch_kernel" not in row.get("Kernel_Name", "") and "qp_pair_kernel" not in row.get("Kernel_Name", ""):
            continue
        tot[row["Counter_Name"]] += float(row["Counter_Value"])
        n[row["Counter_Name"]] += 1
res = {k: v / max(n[k], 1) for k, v in tot.items()}
d = dict(per_dispatch=res)
g = lambda k: res.get(k, float("nan"))
d["derived"] = {
    "l2_read_latency_cycles": g("TCP_TCC_READ_REQ_LATENCY_sum") / g("TCP_TCC_READ_REQ_sum"),
    "l1_hit_rate": 1 - g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum"),
    "l2_hit_rate": g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")),
    "wave_wait_frac": g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"),
    "wave_active_vmem_frac": g("SQ_ACTIVE_INST_VMEM") / g("SQ_WAVE_CYCLES"),
    "wave_active_lds_frac": g("SQ_ACTIVE_INST_LDS") / g("SQ_WAVE_CYCLES"),
    "wave_active_valu_frac": g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"),
    "vmem_level_per_wave_cycle": g("SQ_INST_LEVEL_VMEM") / g("SQ_WAVE_CYCLES"),
    "lds_level_per_wave_cycle": g("SQ_INST_LEVEL_LDS") / g("SQ_WAVE_CYCLES"),
    "vmem_latency_cycles": g("SQ_INST_LEVEL_VMEM") / g("SQ_INSTS_VMEM_RD"),
    "lds_latency_cycles": g("SQ_INST_LEVEL_LDS") / g("SQ_INSTS_LDS"),
}
json.dump(d, open(os.path.join(O, "summary.json"), "w"), indent=1)
print(json.dumps(d, indent=1))
