#!/bin/bash
# quick GPU iteration: gpu tests, phase timing, short bench.  usage: tools/quick.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-quick}"; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 200 python tools/phase_timing.py run 65536 3 > "$O/phase.json" 2> "$O/phase.err" || { echo phase failed; tail -5 "$O/phase.err"; exit 1; }
python -c "import json;d=json.load(open('$O/phase.json'));print(d['cycles_per_solve_step'], d['cycles_per_iter'], d['iters_per_solve'], d['schedule'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -5 "$O/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('solves/s', d['value'], 'frac', d['roofline']['frac'], d['admm_iters'])"
# optional ablation libs: tools/libmpcqp_timing_<NAME>.so -> phase timing each
for L in tools/libmpcqp_timing_*.so; do
  [ -f "$L" ] || continue
  N=$(basename $L .so)
  MPCQP_TIMING_LIB=$R/$L timeout -k 10 200 python tools/phase_timing.py run 65536 3 > "$O/$N.json" 2> "$O/$N.err" || { echo "$N failed"; tail -5 "$O/$N.err"; exit 1; }
  echo "$N: $(python -c "import json;d=json.load(open('$O/$N.json'));print(d['cycles_per_solve_step'], d['cycles_per_iter'])")"
done
