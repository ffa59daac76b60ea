#!/bin/bash
# GPU tests with the in-tree library, then A/B of library builds (10-step bench, alternating).
# usage: tools/ab_libs10.sh <tag> <rounds> lib1.so lib2.so ...
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-ab}"; mkdir -p "$O"; cd "$R"
N=${2:-1}; shift 2
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" "$O/pytest.log" | tail -30; exit 1; }
tail -1 "$O/pytest.log"
fi
for r in $(seq 1 $N); do
  for L in "$@"; do
    tag=$(basename $L .so)
    MPCQP_LIBRARY=$R/$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-10} --warmup 3 > "$O/${tag}_$r.json" 2> "$O/${tag}_$r.err" || { echo "$tag failed"; tail -5 "$O/${tag}_$r.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/${tag}_$r.json'));print('$tag', round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', round(d['admm_iters']['mean'],2))"
  done
done
