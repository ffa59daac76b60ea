#!/bin/bash
# A/B of kernel variants by environment: each argument is "tag:ENV=val,ENV=val" (empty env: the
# default).  Bench at N = 40 delta-v and N = 40 continuous acceleration (--nx 40), 10 steps after 3.
#   usage: tools/ab_modes.sh <outtag> "w1:MPCQP_WAVES=1" "m2:MPCQP_WAVES=3,MPCQP_W0DIAG=0" ...
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-abm}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
shift
for cfg in "40 --dv" "20"; do
  set -- $cfg; ctag=n$1$2
  for spec in $MODES; do
    tag=${spec%%:*}; envs=${spec#*:}
    env_args=$(echo "$envs" | tr ',' ' ')
    env $env_args timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-legs --steps 10 --warmup 3 --nx $cfg > "$O/${ctag}_$tag.json" 2> "$O/${ctag}_$tag.err" || { echo "$ctag $tag failed"; tail -5 "$O/${ctag}_$tag.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${ctag}_$tag.json'));print('$ctag $tag', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],3), d['schedule']['waves_per_cu'])"
  done
done
