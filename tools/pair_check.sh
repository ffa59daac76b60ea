#!/bin/bash
# Kernel-variant check: parity tests of the two-wave kernel (MPCQP_WAVES=2) and of the matrix-
# operand prefetch (MPCQP_MATPF=1), then the bench A/B of the four variants at N = 20 and N = 40
# delta-v.   usage: tools/pair_check.sh <tag> [steps] [variants...]  (variant = "<waves><pf>", e.g. 10 21)
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-pair}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
K=${2:-10}; shift 2
V=${@:-10 11 20 21}
for v in $V; do
  w=${v:0:1}; f=${v:1:1}
  [ "$v" = "10" ] && continue
  MPCQP_WAVES=$w MPCQP_MATPF=$f timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_random_structures.py -x -v --timeout 120 --timeout-method thread > "$O/pytest_$v.log" 2>&1; rc=$?
  echo "pytest variant $v: $(tail -1 $O/pytest_$v.log)"; grep -E "FAILED|Error" "$O/pytest_$v.log" | head -5
  [ $rc -eq 0 ] || exit 1
done
for cfg in "20" "40 --dv"; do
  set -- $cfg; tag=n$1$2
  for v in $V; do
    w=${v:0:1}; f=${v:1:1}
    MPCQP_WAVES=$w MPCQP_MATPF=$f timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-legs --steps $K --warmup 3 --nx $cfg > "$O/${tag}_$v.json" 2> "$O/${tag}_$v.err" || { echo "bench $tag $v failed"; tail -5 "$O/${tag}_$v.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${tag}_$v.json'));print('$tag $v', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],3), d['status_counts'], d['schedule'])"
  done
done
