#!/bin/bash
# Kernel-trace profile of the default bench workload (run on the GPU box).
# usage: tools/profile_run.sh <tag>   -> gpurun_out/prof_<tag>/...
set -o pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err
