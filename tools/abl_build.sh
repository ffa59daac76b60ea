#!/bin/bash
# Fixed-work ablation libraries (125 ADMM iterations per solve, no checks; each drops one piece of
# the iteration -- results are meaningless, only the time counts).  Built here, run on the box with
# tools/ab_libs.sh.   usage: tools/abl_build.sh
# (round 5: the "no solve steps" variant is gone -- its one run hung the card in round 4 and no
# mechanism for it was found in its code; it is not worth a strike to re-run)
export MPCQP_DIAGNOSTICS=1  # the MPCQP_* overrides below are diagnostics (symbolic.hpp diag_env)
set -e
cd "$(dirname "$0")/.."
S="mpc_arpo_project_amd/csrc"
SRC="$S/engine.hip $S/closed_loop.hip $S/estimation.hip $S/symbolic.cpp $S/lds_layout.cpp $S/emulate.cpp"
build() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -DMPCQP_FIXED_WORK "$@" $SRC -o "tools/ab/$TAG.so"
}
TAG=fw_base build &
TAG=fw_nodiag build -DMPCQP_ABL_NODIAG &
TAG=fw_norhs build -DMPCQP_ABL_NORHS &
TAG=fw_noupd build -DMPCQP_ABL_NOUPD &
wait
TAG=fw_novec build -DMPCQP_ABL_NODIAG -DMPCQP_ABL_NORHS -DMPCQP_ABL_NOUPD &
TAG=fw_noscale build -DMPCQP_ABL_NOSCALE &
TAG=fw_nofac build -DMPCQP_ABL_NOFAC &
wait
ls -la tools/ab/fw_*.so
