#!/bin/bash
# A/B of library builds with 1 and 2 shards per GPU (20-step bench).  usage: tools/ab_split1.sh <tag> lib...
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-ab}"; mkdir -p "$O"; cd "$R"; shift
for sp in 1 2; do
for L in "$@"; do
  tag=$(basename $L .so)_s$sp
  MPCQP_LIBRARY=$R/$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --split $sp > "$O/$tag.json" 2> "$O/$tag.err" || { echo "$tag failed"; tail -5 "$O/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'step ms', round(d['ms_per_step'],2), 'iters', round(d['admm_iters']['mean'],2), d['schedule']['waves_per_cu'])"
done
done
