#!/bin/bash
# Round-5 profile evidence on one GPU box (run from the repo root through gpurun), in two parts so
# each call stays well inside its time limit:
#   tools/profile_r5.sh a <tag>: rocprofv3 kernel trace + stats of the default bench (no legs), the
#       N = 40 delta-v bench (config 3) and the continuous-time loop (config 4); calibrated PMC
#       FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md HBM section) of the
#       default workload
#   tools/profile_r5.sh b <tag>: the same PMC passes for N = 40 delta-v, N = 40 continuous
#       acceleration and the continuous-time loop; the SQ LDS counters of N = 20 and N = 40 delta-v
#   tools/profile_r5.sh d <tag>: calibration + PMC passes of BASELINE config 2 (B = 1,024, N = 20)
#   tools/profile_r5.sh c <tag>: the calibration, trace and PMC passes of the continuous-time loop
#       alone (after a change of its layout, e.g. --cont-split)
# Outputs under gpurun_out/<tag>/; tools/profile_post.py turns them into profiles/current/*.json.
set -o pipefail
PART=$1; TAG=${2:-prof_r5}
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-legs"
pmc() {  # pmc <name> <bench args...>: calibrated FETCH_SIZE + WRITE_SIZE passes of one workload
  local n=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_$n" -o run --output-format csv -- "$@" > "$O/bench_fetch_$n.json" 2> "$O/bench_fetch_$n.err" || { echo "fetch $n failed"; tail -3 "$O/bench_fetch_$n.err"; exit 1; }
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d "$O/write_$n" -o run --output-format csv -- "$@" > "$O/bench_write_$n.json" 2> "$O/bench_write_$n.err" || { echo "write $n failed"; tail -3 "$O/bench_write_$n.err"; exit 1; }
  echo "pmc $n ok"
}
calib() {
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_fetch" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_fetch.log" 2>&1 || { echo calib fetch failed; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_write" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_write.log" 2>&1 || { echo calib write failed; exit 1; }
  echo calib ok
}
if [ "$PART" = d ]; then  # config 2: B = 1,024, N = 20, one stream
  calib
  pmc c2 $B --batch 1024 --split 1
elif [ "$PART" = c ]; then
  calib
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_cont" -o run -- python3 $R/bench.py --continuous --steps 5 --warmup 1 > "$O/bench_cont.json" 2> "$O/trace_cont.err" || { echo cont trace failed; tail -5 "$O/trace_cont.err"; exit 1; }
  echo "trace_cont: $(head -c 200 $O/bench_cont.json)"
  pmc cont python3 $R/bench.py --continuous --steps 5 --warmup 1
elif [ "$PART" = a ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_fetch" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_fetch.log" 2>&1 || { echo calib fetch failed; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_write" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_write.log" 2>&1 || { echo calib write failed; exit 1; }
  echo calib ok
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- $B > "$O/bench.json" 2> "$O/trace.err" || { echo trace failed; tail -5 "$O/trace.err"; exit 1; }
  echo "trace: $(head -c 200 $O/bench.json)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace40" -o run -- $B --nx 40 --dv > "$O/bench_n40dv.json" 2> "$O/trace40.err" || { echo n40 trace failed; tail -5 "$O/trace40.err"; exit 1; }
  echo "trace40: $(head -c 200 $O/bench_n40dv.json)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_cont" -o run -- python3 $R/bench.py --continuous --steps 5 --warmup 1 > "$O/bench_cont.json" 2> "$O/trace_cont.err" || { echo cont trace failed; tail -5 "$O/trace_cont.err"; exit 1; }
  echo "trace_cont: $(head -c 200 $O/bench_cont.json)"
  pmc n20 $B
else
  pmc n40dv $B --nx 40 --dv
  pmc n40 $B --nx 40
  pmc cont python3 $R/bench.py --continuous --steps 5 --warmup 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/sq20" -o run --output-format csv -- $B --steps 5 --warmup 2 > "$O/sq20.json" 2> "$O/sq20.err" || { echo sq20 failed; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/sq40" -o run --output-format csv -- $B --nx 40 --dv --steps 5 --warmup 2 > "$O/sq40.json" 2> "$O/sq40.err" || { echo sq40 failed; exit 1; }
  echo sq ok
fi
