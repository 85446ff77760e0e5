#!/bin/bash
# Link an experiment libdsx with the fused-pass objects (dsx_bm, every radius + dispatch) rebuilt under
# extra flags; the other objects come from the in-tree build/.
# usage: bash tools/variant_bm.sh <name> <flags...>  -> tools/explib/libdsx_<name>.so
set -e
N=$1; shift
C=/root/repo/depthestimation_amd/csrc
T=/tmp/varbm_$N
rm -rf $T && cp -rp $C/build $T
for r in 0 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DDSX_RADIUS=$r "$@" -c $C/dsx_bm.hip -o $T/dsx_bm_r$r.o &
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -c $C/dsx_bm.hip -o $T/dsx_bm_dispatch.o &
wait
mkdir -p /root/repo/tools/explib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /root/repo/tools/explib/libdsx_$N.so $T/dsx_*.o -ldl
rm -rf $T
