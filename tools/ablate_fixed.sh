#!/bin/bash
# Fixed-work timing ablations of the product kernel (no s_memtime instrumentation): every build has
# EXP_NOCHECK (125 ADMM iterations per solve, no termination checks), plus one EXP_* skip flag; the
# kernel time differences give the real per-iteration cost of each phase.
#   tools/ablate_fixed.sh build            (container: compiles tools/abl/libmpcqp_<V>.so)
#   tools/ablate_fixed.sh run <tag>        (GPU box: bench each, gpurun_out/<tag>/)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
VARIANTS="${ABL_VARIANTS:-base SKIP_RHS SKIP_FWD SKIP_DIAG SKIP_BWD SKIP_UPDATE NO_RECLOAD}"
if [ "$1" = build ]; then
  mkdir -p "$R/tools/abl"; C="$R/mpc_arpo_project_amd/csrc"
  for v in $VARIANTS; do
    F="-DEXP_NOCHECK"; [[ $v == *CHECK_NOEXIT* ]] && F=""
    [ $v != base ] && for x in ${v//+/ }; do F="$F -DEXP_${x/@/=}"; done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -DMPCQP_ONLY_SMALL $F \
      $C/engine.hip $C/closed_loop.hip $C/estimation.hip $C/symbolic.cpp $C/lds_layout.cpp $C/emulate.cpp \
      -o "$R/tools/abl/libmpcqp_$v.so" 2>&1 | grep -v hip-link &
  done
  wait; ls -la "$R/tools/abl"
  exit 0
fi
O="$R/gpurun_out/${2:-ablfix}"; mkdir -p "$O"; cd "$R"
for v in $VARIANTS; do
  MPCQP_LIBRARY=$R/tools/abl/libmpcqp_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > "$O/$v.json" 2> "$O/$v.err" || { echo "$v failed"; tail -5 "$O/$v.err"; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('$O/$v.json'));print(d['roofline']['kernel_ms_per_launch'], d['admm_iters']['mean'])")"
done
