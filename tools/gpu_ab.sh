#!/bin/bash
# GPU tests, then an A/B of env variants on the default bench (10 steps).  usage:
#   tools/gpu_ab.sh <tag> "NAME=ENV" ...
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-gab}"; mkdir -p "$O"; cd "$R"; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" "$O/pytest.log" | tail -30; exit 1; }
tail -1 "$O/pytest.log"
for v in "$@"; do
  N=${v%%=*}; E=${v#*=}
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-10} --warmup 3 > "$O/$N.json" 2> "$O/$N.err" || { echo "$N failed"; tail -5 "$O/$N.err"; exit 1; }
  echo "$N $(python -c "import json;d=json.load(open('$O/$N.json'));print(round(d['value']), round(d['roofline']['kernel_ms_per_launch'],2), d['admm_iters']['mean'], d['schedule'])")"
done
