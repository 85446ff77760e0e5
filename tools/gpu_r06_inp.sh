#!/bin/bash
# round 6: the OpenCV-form hole filling on the GPU (tests against oracle/telea_cv.c), timings, traces
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inpaint.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_inp6.log 2>&1
rc=$?; echo "inpaint tests rc=$rc"; grep -E "FAIL|Error|error" gpurun_out/t_inp6.log | tail -20; tail -1 gpurun_out/t_inp6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/inpaint_prof.py 20 c2 2>&1 | grep -v amdgpu > gpurun_out/r06_inpaint_times.txt || exit 1
timeout -k 10 180 python tools/inpaint_prof.py 5 c4 2>&1 | grep -v amdgpu >> gpurun_out/r06_inpaint_times.txt || exit 1
cat gpurun_out/r06_inpaint_times.txt
for c in ${CFGS:-c2}; do
  DSX_INPAINT_TRACE=1 timeout -k 10 120 python tools/inpaint_prof.py 1 $c > gpurun_out/trace_$c.txt 2>&1 || exit 1
done
