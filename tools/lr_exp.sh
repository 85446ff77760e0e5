#!/bin/bash
# GPU side of the LR-pass cost split: time the C2 shape (uniqueness x LR) with the in-tree library
# and each experiment build depthestimation_amd/exp/libdsx_e<N>.so (tools/exp_build.sh N ...).
# usage: bash tools/lr_exp.sh <tag> <N...>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  echo "base $(timeout -k 5 120 python3 tools/lr_cost.py --config ${CFG:-c2} --iters 300)" | tee -a $O/lr_exp.txt || exit 1
  for e in "$@"; do
    echo "e$e $(DSX_LIB=$GRAFT_REPO_ROOT/depthestimation_amd/exp/libdsx_e$e.so timeout -k 5 120 python3 tools/lr_cost.py --config ${CFG:-c2} --iters 300)" | tee -a $O/lr_exp.txt || exit 1
  done
done
