#!/bin/bash
# Hole-filling GPU tests, then a rocprofv3 kernel trace of tools/inpaint_prof.py (C4 map).
# usage: bash tools/gpu_inpaint_check.sh <tag>
set -o pipefail
T=${1:-inp}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_inpaint.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/inpaint_prof.py 20 ${CFG:-c4} > $O/log.txt 2>&1
rc=$?; grep median $O/log.txt; exit $rc
