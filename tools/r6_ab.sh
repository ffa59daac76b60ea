#!/bin/bash
# Round-6 A/B on one box: the headline bench (no legs, no CPU baseline) alternating over variants
#   "tag:ENV=val,ENV=val|extra bench args"  (MPCQP_LIBRARY=<repo path> selects another build; empty
#   env = the in-tree library; extra args e.g. --batch 131072 --steps 10)
#   usage: tools/r6_ab.sh <outtag> <rounds> variant...
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-r6ab}"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
N=${2:-1}; shift 2
export MPCQP_DIAGNOSTICS=1
for r in $(seq 1 $N); do
  for spec in "$@"; do
    tag=${spec%%:*}; rest=${spec#*:}
    envs=${rest%%|*}; args=""
    [[ "$rest" == *"|"* ]] && args=${rest#*|}
    env_args=$(echo "$envs" | tr ',' ' ' | sed "s#MPCQP_LIBRARY=#MPCQP_LIBRARY=$R/#")
    env $env_args timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-legs $AB_ARGS $args > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err" || { echo "$tag failed"; tail -5 "$O/${tag}_$r.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${tag}_$r.json'));s=d['schedule'];print('$tag', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],3), 'Mit/s', round(d['roofline']['admm_iters_timed']/d['ms_per_step']/d['steps']/1e3,2), 'regs', s.get('kernel_regs'), 'scratch', s.get('kernel_scratch_bytes'))"
  done
done
