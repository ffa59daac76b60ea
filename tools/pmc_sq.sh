#!/bin/bash
# SQ counter pass (issue / wait / LDS breakdown) of a short bench run; one counter group per pass.
set -o pipefail
set -e
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/pmc_sq"
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$O/p1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$O/b1.json" 2> "$O/b1.err"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d "$O/p2" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$O/b2.json" 2> "$O/b2.err"
