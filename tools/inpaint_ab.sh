#!/bin/bash
# Hole filling A/B on the C4 map: per-layer launches (default) against the persistent march
# (DSX_INPAINT_L0=0) at several grid sizes (DSX_INPAINT_RB), twice in alternating order.
# usage: bash tools/inpaint_ab.sh <tag>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_inpaint.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  echo "default $(timeout -k 5 60 python3 tools/inpaint_prof.py 40)" | tee -a $O/ab.txt || exit 1
  for rb in 256 128 64 32; do
    echo "L0=0 RB=$rb $(DSX_INPAINT_L0=0 DSX_INPAINT_RB=$rb timeout -k 5 60 python3 tools/inpaint_prof.py 40)" | tee -a $O/ab.txt || exit 1
  done
done
