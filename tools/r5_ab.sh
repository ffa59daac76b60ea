#!/bin/bash
# Round-5 A/B on one box: (1) the given pytest files; (2) the headline bench (no legs, no CPU
# baseline) alternating over variants "tag:ENV=val,ENV=val" (MPCQP_LIBRARY=<repo path> selects
# another build; empty env = the in-tree library).
#   usage: tools/r5_ab.sh <outtag> <rounds> "<pytest files or -" variant...
# A pytest assertion failure (rc 1) does not stop the A/B; anything else (fault, abort, time
# limit) ends the call there.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-r5ab}"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
N=${2:-1}; TESTS="$3"; shift 3
if [ "$TESTS" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
  rc=$?
  tail -3 "$O/pytest.log"
  grep -E "^FAILED|Error" "$O/pytest.log" | head -10
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
fi
export MPCQP_DIAGNOSTICS=1
for r in $(seq 1 $N); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env_args=$(echo "$envs" | tr ',' ' ' | sed "s#MPCQP_LIBRARY=#MPCQP_LIBRARY=$R/#")
    env $env_args timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-legs $AB_ARGS > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err" || { echo "$tag failed"; tail -5 "$O/${tag}_$r.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${tag}_$r.json'));s=d['schedule'];print('$tag', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],3), 'cold', round(d['cold']['value']), 'regs', s.get('kernel_regs'), 'scratch', s.get('kernel_scratch_bytes'))"
  done
done
