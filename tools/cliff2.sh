#!/bin/bash
# Threshold of the register cliff: pad builds around 448 allocated registers, one
# stream and two streams, status counts against the unpadded build.  usage: tools/cliff2.sh <tag>
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-cliff2}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for p in 0 28 32 36 38 40 44 56; do
  for s in 1 2; do
    MPCQP_LIBRARY=$R/tools/ab/pad$p.so timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-legs --batch 16384 --steps 3 --warmup 2 --split $s > "$O/pad${p}_s$s.json" 2> "$O/pad${p}_s$s.err" || { echo "pad$p s$s failed"; tail -5 "$O/pad${p}_s$s.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/pad${p}_s$s.json'));print('pad$p split$s', round(d['value']), 'iters', round(d['admm_iters']['mean'],3), d['status_counts'])"
  done
done
MPCQP_LIBRARY=$R/tools/ab/pad56.so timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$O/pytest_pad56.log" 2>&1; echo "pytest pad56 rc=$?"; tail -3 "$O/pytest_pad56.log"
