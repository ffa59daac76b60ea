#!/bin/bash
# One GPU-box pass: gpu tests, smoke, the default bench (CPU baseline + config-3 leg), the
# continuous-time (config 4) bench.  usage: tools/gpu_check.sh <tag>   -> gpurun_out/<tag>/...
#   GC_SKIP_TESTS=1 skips pytest; GC_CONT_STEPS sets the config-4 timed periods (default 5)
set -o pipefail
TAG=${1:-check}
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$R"
if [ -z "$GC_SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" "$O/pytest.log" | tail -30; exit 1; }
  tail -1 "$O/pytest.log"
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; cat "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -20 "$O/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value']), d['admm_iters'], 'frac', round(d['roofline']['frac'],4), 'config3', round(d['config3'].get('value',0)), 'n40_accel', round(d['n40_accel'].get('value',0)), 'config4', round(d['config4'].get('value',0)), 'cpu', round(d.get('cpu_baseline',{}).get('value',0)))"
timeout -k 10 600 python bench.py --continuous --steps ${GC_CONT_STEPS:-5} --warmup 1 > "$O/bench_cont.json" 2> "$O/bench_cont.err" || { echo cont bench failed; tail -20 "$O/bench_cont.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_cont.json'));print('continuous', round(d['value']), d['period_split_ms'], d['admm_iters'])"
