#!/bin/bash
# Register-pressure builds vs the product (the r03 "cliff"): SGPR spills to memory
# (_nosv), AGPR pads, VGPR pads; one stream, status counts.   usage: tools/cliff3.sh <tag> libs...
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-cliff3}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
shift
for L in "$@"; do
  MPCQP_LIBRARY=$R/tools/ab/$L.so timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-legs --batch 16384 --steps 3 --warmup 2 --split 1 > "$O/$L.json" 2> "$O/$L.err" || { echo "$L failed"; tail -5 "$O/$L.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$L.json'));print('$L', round(d['value']), 'iters', round(d['admm_iters']['mean'],3), d['status_counts'])"
done
