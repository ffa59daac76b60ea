#!/bin/bash
# Warm lockstep parity test (tests/test_gpu_scale_parity.py) against several library builds / plan
# environments; prints each run's per-step agreement line.
#   tools/lockstep_variants.sh <tag> "ENV=.. lib.so" ...
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-lsv}"; mkdir -p "$O"; cd "$R"; shift
i=0
for spec in "$@"; do
  i=$((i+1))
  env $spec timeout -k 10 300 python -u -m pytest tests/test_gpu_scale_parity.py -k lockstep -x -q -s --timeout 280 --timeout-method thread > "$O/v$i.log" 2>&1
  rc=$?
  echo "[$spec] rc=$rc $(grep -o 'per-step status agreement.*' "$O/v$i.log" | head -1)"
  [ $rc -gt 1 ] && exit 1
done
exit 0
