#!/bin/bash
# The > 190-AGPR shard-overlap cliff: the product kernel with 0 / 24 / 40 / 56
# extra AGPRs held live (tools/ab/pad*.so, -DMPCQP_PAD_AGPR, nothing else changed): default bench
# per build, then a rocprofv3 kernel trace of pad0 and pad56 (per-dispatch start / end of the two
# shards' launches on their two streams).   usage: tools/cliff.sh <tag>
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-cliff}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for p in 0 24 40 56; do
  MPCQP_LIBRARY=$R/tools/ab/pad$p.so timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-legs --steps 10 --warmup 3 > "$O/pad$p.json" 2> "$O/pad$p.err" || { echo "pad$p failed"; tail -5 "$O/pad$p.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pad$p.json'));print('pad$p', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2))"
done
for p in 0 56; do
  MPCQP_LIBRARY=$R/tools/ab/pad$p.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_pad$p" -o run -- python3 $R/bench.py --no-cpu-baseline --no-legs --steps 10 --warmup 3 > "$O/trace_pad$p.json" 2> "$O/trace_pad$p.err" || { echo "trace pad$p failed"; tail -5 "$O/trace_pad$p.err"; exit 1; }
  echo "trace pad$p ok"
done
