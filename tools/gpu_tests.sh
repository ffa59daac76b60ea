#!/bin/bash
# GPU tests only (optionally a -k filter).  usage: tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-tests}"; mkdir -p "$O"; cd "$R"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${K[@]}" > "$O/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|agree|checked|optima|status" "$O/pytest.log" | tail -60
exit $rc
