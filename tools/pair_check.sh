#!/bin/bash
# Two-wave kernel check (MPCQP_WAVES=2): parity tests, then the bench A/B against the one-wave
# kernel at N = 20 and N = 40 delta-v.   usage: tools/pair_check.sh <tag> [steps]
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-pair}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
K=${2:-10}
MPCQP_WAVES=2 timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_random_structures.py -x -v --timeout 120 --timeout-method thread > "$O/pytest_w2.log" 2>&1; rc=$?
tail -3 "$O/pytest_w2.log"; grep -E "FAILED|Error" "$O/pytest_w2.log" | head -5
[ $rc -eq 0 ] || exit 1
for cfg in "20" "40 --dv"; do
  set -- $cfg; tag=n$1$2
  for w in 1 2; do
    MPCQP_WAVES=$w timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-legs --steps $K --warmup 3 --nx $cfg > "$O/${tag}_w$w.json" 2> "$O/${tag}_w$w.err" || { echo "bench $tag w$w failed"; tail -5 "$O/${tag}_w$w.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${tag}_w$w.json'));print('$tag w$w', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],3), d['status_counts'], d['schedule'])"
  done
done
