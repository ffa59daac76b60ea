#!/bin/bash
# round 6: the bitwise engine-vs-hybrid test, then the hybrid sweep runs of one case
O=gpurun_out/$1; mkdir -p $O; CASE=${2:-radial20}; N=${3:-1024}
timeout -k 10 600 python -u -m pytest tests/test_gpu_hybrid.py -x -v --timeout 300 --timeout-method thread > $O/pytest_hybrid.log 2>&1; rc=$?
tail -8 $O/pytest_hybrid.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 900 python -u tools/parity_floor.py --case $CASE --n $N --hybrid-only > $O/hybrid_$CASE.json 2> $O/hybrid_$CASE.err || { echo "parity_floor failed"; tail -20 $O/hybrid_$CASE.err; exit 1; }
cat $O/hybrid_$CASE.err | tail -6; cat $O/hybrid_$CASE.json
