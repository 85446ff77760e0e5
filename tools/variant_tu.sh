#!/bin/bash
# Link an experiment libdsx with ONE translation unit rebuilt under extra flags (the other objects come
# from the in-tree build/).  usage: bash tools/variant_tu.sh <name> <tu: dsx_post|dsx_api|...> <flags...>
# -> tools/explib/libdsx_<name>.so (OUTDIR overrides; SRC=<file> compiles another copy of the TU)
set -e
N=$1; TU=$2; shift 2
C=/root/repo/depthestimation_amd/csrc
T=/tmp/vartu_$N
rm -rf $T && cp -rp $C/build $T
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I$C "$@" -c ${SRC:-$C/$TU.hip} -o $T/$TU.o
OUT=${OUTDIR:-/root/repo/tools/explib}; mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libdsx_$N.so $T/dsx_*.o -ldl
