#!/bin/bash
# GPU tests + default bench + small sweep (radial and in-track).  usage: tools/r02_check.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-chk}"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" "$O/pytest.log" | tail -30; exit 1; }
grep -E "passed|agree|checked|optima|disagreeing" "$O/pytest.log" | tail -20
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; cat "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 500 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 python -m mpc_arpo_project_amd.sweep --scenario radial --seeds 16 --ics 1024 > "$O/sweep_radial.json" 2> "$O/sweep_radial.err" || { echo sweep failed; tail -20 "$O/sweep_radial.err"; exit 1; }
cat "$O/sweep_radial.json"
timeout -k 10 300 python -m mpc_arpo_project_amd.sweep --scenario in_track --nx 40 --no-reject --noise none --seeds 1 --ics 4096 > "$O/sweep_intrack.json" 2> "$O/sweep_intrack.err" || { echo sweep it failed; tail -20 "$O/sweep_intrack.err"; exit 1; }
cat "$O/sweep_intrack.json"
