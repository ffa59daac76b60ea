#!/bin/bash
# Profile evidence at HEAD (GPU box): default bench with the CPU baseline; rocprofv3 kernel trace of
# the default workload; PMC passes (FETCH_SIZE / WRITE_SIZE with calibration, SQ LDS counters); the
# N=40 impulsive delta-v bench (BASELINE config 3) with its kernel trace; the continuous-time loop
# (config 4) with its kernel trace.   usage: tools/profile.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-prof}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-legs"
timeout -k 10 400 python3 $R/bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -5 "$O/bench.err"; exit 1; }
echo "bench: $(head -c 300 $O/bench.json)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- $B > "$O/trace_bench.json" 2> "$O/trace.err" || { echo trace failed; tail -5 "$O/trace.err"; exit 1; }
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_fetch" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_fetch.log" 2>&1 || { echo calib fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_write" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_write.log" 2>&1 || { echo calib write failed; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- $B > "$O/bench_fetch.json" 2> "$O/bench_fetch.err" || { echo fetch failed; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- $B > "$O/bench_write.json" 2> "$O/bench_write.err" || { echo write failed; exit 1; }
echo pmc traffic ok
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d "$O/sq1" -o run --output-format csv -- $B --steps 5 --warmup 2 > "$O/sq1.json" 2> "$O/sq1.err" || { echo sq1 failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE -d "$O/sq2" -o run --output-format csv -- $B --steps 5 --warmup 2 > "$O/sq2.json" 2> "$O/sq2.err" || { echo sq2 failed; exit 1; }
echo sq ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace40" -o run -- $B --nx 40 --dv > "$O/bench40.json" 2> "$O/bench40.err" || { echo n40 failed; tail -5 "$O/bench40.err"; exit 1; }
echo "n40: $(head -c 300 $O/bench40.json)"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/sq40" -o run --output-format csv -- $B --nx 40 --dv --steps 5 --warmup 2 > "$O/sq40.json" 2> "$O/sq40.err" || { echo sq40 failed; exit 1; }
echo sq40 ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_cont" -o run -- python3 $R/bench.py --continuous --steps 5 --warmup 1 > "$O/bench_cont.json" 2> "$O/bench_cont.err" || { echo continuous trace failed; tail -5 "$O/bench_cont.err"; exit 1; }
echo "continuous: $(head -c 300 $O/bench_cont.json)"
