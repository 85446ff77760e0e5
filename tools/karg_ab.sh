#!/bin/bash
# LR-pass kernarg reload (DSX_KARG) A/B: in-tree library (reload on) against exp/libdsx_e0.so (built
# with -DDSX_KARG=0), C4, C2 and C3 shapes (tools/lr_cost.py), two alternating repetitions each.
# usage: bash tools/karg_ab.sh <tag>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_sgbm_lr.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for c in c4 c2 c3; do
  CFG=$c bash tools/lr_exp.sh $1 0 || exit 1
done
