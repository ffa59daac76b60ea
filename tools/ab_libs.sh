#!/bin/bash
# A/B of engine builds on one box: the default bench (no CPU baseline, no config-3 leg) with each
# library, alternating.  Extra bench flags in AB_ARGS (e.g. AB_ARGS="--split 1 --steps 10").
# usage: tools/ab_libs.sh <tag> <rounds> lib1.so lib2.so ...   (paths relative to the repo root)
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-ab}"; mkdir -p "$O"; cd "$R"
N=${2:-1}; shift 2
for r in $(seq 1 $N); do
  for L in "$@"; do
    tag=$(basename $L .so)
    MPCQP_LIBRARY=$R/$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs $AB_ARGS > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err" || { echo "$tag failed"; tail -5 "$O/${tag}_$r.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/${tag}_$r.json'));print('$tag', round(d['value']), 'waves/cu', d['schedule']['waves_per_cu'], 'lds', d['schedule']['lds_bytes'], 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],2), 'cold', round(d['cold']['value']), 'cold kernel ms', round(d['cold']['kernel_ms_per_launch'],2))"
  done
done
