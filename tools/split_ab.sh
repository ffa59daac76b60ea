#!/bin/bash
# Headline bench (20 steps after 5, no legs, no CPU baseline) at several shard counts.
#   usage: tools/split_ab.sh <tag> [splits...]
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-split}"; mkdir -p "$O"; shift; cd "$R"
for s in ${@:-2 3 4}; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-legs --split $s > "$O/split$s.json" 2> "$O/split$s.err" || { echo "split $s failed"; tail -5 "$O/split$s.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/split$s.json'));print('split $s', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_launch'],2), round(d['admm_iters']['mean'],3))"
done
