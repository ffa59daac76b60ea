#!/bin/bash
# GPU parity tests of the engine + the default bench; prints the headline and each leg's step time
# against its per-launch kernel time (overlap of the two shards).  usage: tools/legs_check.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-legs}"; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 600 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -20 "$O/bench.err"; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("bench", round(d["value"]), round(d["ms_per_step"], 2), round(d["roofline"]["kernel_ms_per_launch"], 2), round(d["roofline"]["frac"], 4))
for k in ("config3", "n40_accel", "config4"):
    x = d[k]
    print(k, round(x["value"]), round(x["ms_per_step"], 1), round(x["roofline"]["kernel_ms_per_launch"], 1), round(x["roofline"]["frac"], 4), x["roofline"]["kernel"])
PY
