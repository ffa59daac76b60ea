#!/bin/bash
# Phase timing of the timing-ablation builds (tools/libmpcqp_timing_*.so), GPU box.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/ablate"; mkdir -p "$O"; cd "$R"
for v in base NO_LADDER NO_LDSREAD NO_RECLOAD ALL; do
  if [ $v = base ]; then L=tools/libmpcqp_timing.so; else L=tools/libmpcqp_timing_$v.so; fi
  MPCQP_TIMING_LIB=$R/$L timeout -k 10 200 python tools/phase_timing.py run 16384 2 > "$O/$v.json" 2> "$O/$v.err" || { echo "$v failed"; tail -5 "$O/$v.err"; exit 1; }
  echo "$v: $(python -c "import json;d=json.load(open('$O/$v.json'));print(d['cycles_per_solve_step'], d['cycles_per_iter'], d['iters_per_solve'])")"
done
