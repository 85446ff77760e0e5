#!/bin/bash
# hole-filling A/B of libdsx builds (tools/inpaint_policy.py, both launch policies), alternating, with
# the inpaint GPU tests on the in-tree build first.  usage: bash tools/gpu_inp_lib_ab.sh <lib> [lib...]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/inp_lib_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_inpaint.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/inp_lib_ab_tests.txt 2>&1 || { tail -20 gpurun_out/inp_lib_ab_tests.txt; exit 1; }
tail -1 gpurun_out/inp_lib_ab_tests.txt
: > $O
for rep in 1 2; do
  for v in "$@" new; do
    if [ $v = new ]; then L=$GRAFT_REPO_ROOT/depthestimation_amd/libdsx.so; else L=$GRAFT_REPO_ROOT/$v; fi
    DSX_LIB=$L timeout -k 10 300 python -u tools/inpaint_policy.py c2 10 -1,0 >> $O 2>&1 || { tail -5 $O; exit 1; }
    DSX_LIB=$L timeout -k 10 300 python -u tools/inpaint_policy.py c4 3 -1,0 >> $O 2>&1 || { tail -5 $O; exit 1; }
  done
done
grep config $O
