#!/bin/bash
# A/B of the solve order (bench --order iters|none) x chaser shards (--split 1|2), alternating on one
# box.  usage (GPU box): tools/ab_order.sh <tag> <rounds>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-ab_order}"; mkdir -p "$O"; cd "$R"
for r in $(seq 1 ${2:-1}); do
  for cfg in "none 2" "iters 2" "iters 1" "none 1"; do
    set -- $cfg; tag="order_$1_split_$2"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --order $1 --split $2 > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err" || { echo "$tag failed"; tail -5 "$O/${tag}_$r.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/${tag}_$r.json'));print('$tag', round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'ms/step', round(d['ms_per_step'],2), 'iters', round(d['admm_iters']['mean'],2))"
  done
done
