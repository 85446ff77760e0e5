#!/bin/bash
# Build experiment variants of libdsx.so (compile-time DSX_EXP bits in dsx_bm.hip) into
# depthestimation_amd/exp/libdsx_e<N>.so, for A/B timing with DSX_LIB=... (dev tool)
set -e
cd "$(dirname "$0")/../depthestimation_amd/csrc"
mkdir -p ../exp
for e in "$@"; do
  make -s -j8 OBJ=build_e$e OUT=../exp FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DDSX_EXP=$e $EXTRA" ../exp/libdsx.so >/dev/null
  mv ../exp/libdsx.so ../exp/libdsx_e$e.so
done
