#!/bin/bash
# Volume-path kernel times: in-tree library against exp/libdsx_e0.so, alternating, configs given.
# usage: bash tools/k2_ab.sh <tag> c4 c2 ...
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  echo "base $(timeout -k 5 120 python3 tools/k2_time.py "$@")" | tee -a $O/k2.txt || exit 1
  echo "e0 $(DSX_LIB=$GRAFT_REPO_ROOT/depthestimation_amd/exp/libdsx_e0.so timeout -k 5 120 python3 tools/k2_time.py "$@")" | tee -a $O/k2.txt || exit 1
done
