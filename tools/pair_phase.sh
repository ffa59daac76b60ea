#!/bin/bash
# Phase timing (tools/phase_timing.py, timing build) of the one- and two-wave kernels at N = 20
# and N = 40, and the bench of both with one shard (--split 1).   usage: tools/pair_phase.sh <tag>
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-pphase}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for nx in 20 40; do
  for w in ${WAVES:-1 2 3}; do
    MPCQP_WAVES=$w timeout -k 10 300 python3 $R/tools/phase_timing.py run 65536 5 3 $nx > "$O/phase_n${nx}_w$w.json" 2> "$O/phase_n${nx}_w$w.err" || { echo "phase n$nx w$w failed"; tail -5 "$O/phase_n${nx}_w$w.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/phase_n${nx}_w$w.json'));print('n$nx w$w', 'kernel ms', round(d['kernel_ms_per_launch'],2), 'iters', round(d['iters_per_solve'],1), {k: round(v) for k,v in d['cycles_per_solve'].items()}, 'per iter', {k: round(v) for k,v in d['cycles_per_iter'].items()})"
  done
done
for w in ${WAVES:-1 2 3}; do
  MPCQP_WAVES=$w timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-legs --steps 10 --warmup 3 --split 1 > "$O/n20_s1_w$w.json" 2> "$O/n20_s1_w$w.err" || { echo "bench s1 w$w failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/n20_s1_w$w.json'));print('n20 split1 w$w', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2))"
done
