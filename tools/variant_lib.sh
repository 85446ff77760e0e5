#!/bin/bash
# Link an experiment libdsx with one fused-pass radius TU rebuilt under extra flags (the other
# objects come from the in-tree build/).  usage: bash tools/variant_lib.sh <name> <radius> <flags...>
# -> tools/explib/libdsx_<name>.so
set -e
N=$1; R=$2; shift 2
C=/root/repo/depthestimation_amd/csrc
T=/tmp/varlib_$N
rm -rf $T && cp -rp $C/build $T
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DDSX_RADIUS=$R "$@" -c ${SRC:-$C/dsx_bm.hip} -o $T/dsx_bm_r$R.o
mkdir -p /root/repo/tools/explib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /root/repo/tools/explib/libdsx_$N.so $T/dsx_*.o -ldl
