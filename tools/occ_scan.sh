#!/bin/bash
# Occupancy scan: the default bench (1 shard) with the LDS allocation padded so that 1..4 instances
# fit a CU (MPCQP_LDS_PAD, diagnostic only).  usage: tools/occ_scan.sh <tag> [lib.so]
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-occ}"; mkdir -p "$O"; cd "$R"
[ -n "$2" ] && export MPCQP_LIBRARY=$R/$2
for pad in 90000 40000 15600 0; do
  MPCQP_LDS_PAD=$pad timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --split 1 > "$O/occ_$pad.json" 2> "$O/occ_$pad.err" || { echo "occ $pad failed"; tail -5 "$O/occ_$pad.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/occ_$pad.json'));print('pad $pad', d['schedule']['waves_per_cu'], 'solves/s', round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', d['admm_iters']['mean'])"
done
