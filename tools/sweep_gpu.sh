#!/bin/bash
# GPU box: gpu tests, then the default bench at several block caps.  usage: tools/sweep_gpu.sh <tag> "M/W M/W ..."
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-sweep}"; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for c in $2; do
  M=${c%/*}; W=${c#*/}
  MPCQP_CAPM=$M MPCQP_CAPW=$W timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > "$O/b_${M}_${W}.json" 2> "$O/b_${M}_$W.err" || { echo "bench $c failed"; tail -5 "$O/b_${M}_$W.err"; exit 1; }
  echo "$c $(python -c "import json;d=json.load(open('$O/b_${M}_${W}.json'));print(round(d['value']), d['schedule'], d['admm_iters']['mean'])")"
done
