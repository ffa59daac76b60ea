#!/bin/bash
# A/B of environment-selected variants of one library on the headline bench (default N = 20,
# 20 steps after 5, no legs, no CPU baseline), alternating for <rounds> rounds.
#   usage: tools/ab_env.sh <outtag> <rounds> "tag:ENV=val,ENV=val" ...  (empty env: the default)
#   extra bench flags in AB_ARGS (e.g. AB_ARGS="--nx 40 --dv")
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-abe}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
N=${2:-1}; shift 2
for r in $(seq 1 $N); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env_args=$(echo "$envs" | tr ',' ' ')
    env $env_args timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-legs $AB_ARGS > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err" || { echo "$tag failed"; tail -5 "$O/${tag}_$r.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${tag}_$r.json'));s=d['schedule'];print('$tag', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],3), 'per_cu', s.get('instances_per_cu'), 'regs', s.get('kernel_regs'), 'lds', s['lds_bytes'], 'steps', s['fwd_steps']+s['bwd_steps'])"
  done
done
