#!/bin/bash
# Hole filling on the C4 map, stream events without a profiler: in-tree library against
# exp/libdsx_e0.so (an earlier build), alternating.  usage: bash tools/inpaint_lib_ab.sh <tag>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
for rep in 1 2 3; do
  echo "base $(timeout -k 5 60 python3 tools/inpaint_prof.py 40)" | tee -a $O/inp.txt || exit 1
  echo "e0 $(DSX_LIB=$GRAFT_REPO_ROOT/depthestimation_amd/exp/libdsx_e0.so timeout -k 5 60 python3 tools/inpaint_prof.py 40)" | tee -a $O/inp.txt || exit 1
done
