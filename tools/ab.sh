#!/bin/bash
# A/B on ONE GPU box (devices differ by several %): alternating default-config bench runs of
# variants given as "NAME=ENV_ASSIGNMENTS" (e.g. "base=" "lpt=MPCQP_LPT=1" "v2=MPCQP_LIBRARY=/path").
#   tools/ab.sh <tag> <rounds> <variant>...
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-ab}"; mkdir -p "$O"; cd "$R"
ROUNDS=${2:-2}; shift 2
for k in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    N=${v%%=*}; E=${v#*=}
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-20} --warmup 3 > "$O/${N}_$k.json" 2> "$O/${N}_$k.err" || { echo "$N failed"; tail -5 "$O/${N}_$k.err"; exit 1; }
    echo "$N #$k $(python -c "import json;d=json.load(open('$O/${N}_$k.json'));print(round(d['value']), round(d['roofline']['kernel_ms_per_launch'],2), d['admm_iters']['mean'])")"
  done
done
