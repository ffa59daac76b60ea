#!/bin/bash
# Round-6 counter study of the N = 20 solve kernel: one counter group per rocprofv3 pass (block
# limits: 8 SQ, 4 TCP, 2 TA, 2 TD, 4 TCC, 2 GRBM), each over a short bench run of the default
# workload.  usage: tools/pmc_study.sh <outtag> [extra bench args]
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-pmcs}"; mkdir -p "$O"; shift
cd /tmp && export TMPDIR=/tmp
P=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
 "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
 "TA_TA_BUSY_sum TA_BUFFER_COALESCED_READ_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
 "TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TCC_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
 "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_LATENCY_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
)
i=0
for c in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $c -d "$O/p$i" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-legs --steps 3 --warmup 1 "$@" > "$O/b$i.json" 2> "$O/b$i.err" || { echo "pass $i failed"; tail -5 "$O/b$i.err"; exit 1; }
  echo "pass $i ok"
done
python3 "$R/tools/pmc_study_sum.py" "$O"
