#!/bin/bash
# PMC passes of the N = 40 impulsive delta-v workload (BASELINE config 3; the two-wave kernel):
# FETCH_SIZE and WRITE_SIZE (separate passes, calibrated as tools/profile.sh) and the SQ LDS
# counters with GRBM_GUI_ACTIVE.   usage: tools/profile40.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-prof40}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-legs --nx 40 --dv"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_fetch" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_fetch.log" 2>&1 || { echo calib fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_write" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_write.log" 2>&1 || { echo calib write failed; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- $B > "$O/bench_fetch.json" 2> "$O/bench_fetch.err" || { echo fetch failed; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- $B > "$O/bench_write.json" 2> "$O/bench_write.err" || { echo write failed; exit 1; }
echo pmc traffic ok
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/sq40" -o run --output-format csv -- $B --steps 5 --warmup 2 > "$O/sq40.json" 2> "$O/sq40.err" || { echo sq40 failed; exit 1; }
echo sq40 ok
