#!/bin/bash
# hole filling: inpaint GPU tests on the in-tree build, a library A/B (default launch policy), and the
# per-step device stamps of the default policy at C2 / C4 (DSX_INPAINT_STAMPS)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/inp3_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_inpaint.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/inp3_tests.txt 2>&1 || { tail -20 gpurun_out/inp3_tests.txt; exit 1; }
tail -1 gpurun_out/inp3_tests.txt
: > $O
for rep in 1 2; do
  for v in "$@" new; do
    if [ $v = new ]; then L=$GRAFT_REPO_ROOT/depthestimation_amd/libdsx.so; else L=$GRAFT_REPO_ROOT/$v; fi
    DSX_LIB=$L timeout -k 10 300 python -u tools/inpaint_policy.py c2 10 0 >> $O 2>&1 || { tail -5 $O; exit 1; }
    DSX_LIB=$L timeout -k 10 300 python -u tools/inpaint_policy.py c4 4 0 >> $O 2>&1 || { tail -5 $O; exit 1; }
  done
done
grep config $O
rm -f gpurun_out/stamps3_c2.txt gpurun_out/stamps3_c4.txt
DSX_INPAINT_STAMPS=$PWD/gpurun_out/stamps3_c2.txt timeout -k 10 300 python -u tools/inpaint_policy.py c2 2 0 > /dev/null 2>&1 || exit 1
DSX_INPAINT_STAMPS=$PWD/gpurun_out/stamps3_c4.txt timeout -k 10 300 python -u tools/inpaint_policy.py c4 1 0 > /dev/null 2>&1 || exit 1
wc -l gpurun_out/stamps3_c*.txt
