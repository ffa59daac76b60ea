#!/bin/bash
# round-6 GPU check: the GPU tests, then the default bench (driver-style), each under its own limit
O=gpurun_out/$1; mkdir -p $O
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], {k:v.get('value') for k,v in d.get('legs',{}).items()})"
