#!/bin/bash
# Default bench (no CPU baseline) with 1-4 concurrent chaser shards per GPU, same box.
# usage: tools/split_scan.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-split}"; mkdir -p "$O"; cd "$R"
for s in 2 3 4 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --split $s > "$O/split${s}_$SECONDS.json" 2> "$O/split$s.err" || { echo "split $s failed"; tail -5 "$O/split$s.err"; exit 1; }
  python -c "import json,glob,os;f=max(glob.glob('$O/split${s}_*.json'),key=os.path.getmtime);d=json.load(open(f));print('split', $s, round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],2))"
done
