#!/bin/bash
# One GPU-box pass: gpu tests, smoke, default bench (with CPU baseline), kernel-trace profile.
# usage: tools/gpu_check.sh <tag>   -> gpurun_out/<tag>/...
set -o pipefail
TAG=${1:-check}
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; cat "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof_bench.err" || { echo prof failed; tail -20 "$O/prof_bench.err"; exit 1; }
cat "$O/prof_bench.json"
find "$O/prof" -name "*stats*"
