#!/bin/bash
# Warm lockstep parity (tests/test_gpu_scale_parity.py -k lockstep) under the planner's copy-row modes
# (MPCQP_COPY_ROWS, symbolic.cpp).  usage (GPU box): LK_MODES="0 1 4" bash tools/lockstep_modes.sh
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -o pipefail
mkdir -p gpurun_out/lk
for m in ${LK_MODES:-0 1 2}; do
  MPCQP_COPY_ROWS=$m timeout -k 10 400 python -u -m pytest tests/test_gpu_scale_parity.py -k lockstep -x -q -s --timeout 380 > gpurun_out/lk/mode$m.log 2>&1
  echo "mode $m rc $?"; grep -E "flips|agreement" gpurun_out/lk/mode$m.log | cut -c1-400
done
