#!/bin/bash
# same-box comparison of bench.py --split values (default bench otherwise).  tools/ab_split.sh <tag> "1 2 4"
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-split}"; mkdir -p "$O"; cd "$R"
for k in 1 2; do
  for S in $2; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --split $S > "$O/s${S}_$k.json" 2> "$O/s${S}_$k.err" || { echo "split $S failed"; tail -5 "$O/s${S}_$k.err"; exit 1; }
    echo "split $S #$k $(python -c "import json;d=json.load(open('$O/s${S}_$k.json'));print(round(d['value']), round(d['roofline']['kernel_ms_per_launch'],2), d['admm_iters']['mean'], round(d['roofline']['frac'],3))")"
  done
done
