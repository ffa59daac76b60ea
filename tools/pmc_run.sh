#!/bin/bash
# PMC passes for profiles/pmc_traffic.json (run on the GPU box from the repo root):
# calibration (FETCH_SIZE, WRITE_SIZE) then the default bench workload, one counter per pass.
set -o pipefail
set -e
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/pmc"
mkdir -p "$O"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_fetch" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_fetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_write" -o run --output-format csv -- "$R/tools/pmc_calib" > "$O/calib_write.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_fetch.json" 2> "$O/bench_fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_write.json" 2> "$O/bench_write.err"
