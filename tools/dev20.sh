#!/bin/bash
# A/B library of the N = 20 product kernel alone (-DMPCQP_DEV20: no other kernel instantiated),
# with the other sources from the product build's objects.  usage: tools/dev20.sh out.so [-D...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/mpc_arpo_project_amd/csrc; O=$R/build/obj; mkdir -p $O
out=$1; shift
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result"
for f in closed_loop.hip estimation.hip host_abi.cpp symbolic.cpp lds_layout.cpp emulate.cpp; do
  o=$O/${f%.*}.o
  [ -f $o ] && [ $o -nt $C/$f ] || $HIPCC -c $C/$f -o $o &
done
tag=$(echo "$@" | md5sum | cut -c1-8)
$HIPCC -DMPCQP_DEV20 "$@" -c $C/engine.hip -o $O/engine_dev20_$tag.o
wait
$HIPCC -shared -o $out $O/engine_dev20_$tag.o $O/closed_loop.o $O/estimation.o $O/host_abi.o $O/symbolic.o $O/lds_layout.o $O/emulate.o
