#!/bin/bash
# Occupancy scan of the headline bench (default shards, 20 steps after 5) for several libraries:
# the LDS allocation padded (MPCQP_LDS_PAD, diagnostic) so that 2, 3 and 4 instances fit a CU.
# usage: tools/occ_ab.sh <tag> lib1.so [lib2.so ...]   -> gpurun_out/<tag>/
export MPCQP_DIAGNOSTICS=1
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-occ}"; mkdir -p "$O"; cd "$R"; shift
for L in "$@"; do
  tag=$(basename $L .so)
  for pad in ${OCC_PADS:-30000 10000 0}; do
    MPCQP_LIBRARY=$R/$L MPCQP_LDS_PAD=$pad timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs > "$O/${tag}_$pad.json" 2> "$O/${tag}_$pad.err" || { echo "$tag $pad failed"; tail -5 "$O/${tag}_$pad.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/${tag}_$pad.json'));print('$tag pad $pad', d['schedule']['waves_per_cu'], 'solves/s', round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', d['admm_iters']['mean'])"
  done
done
