#!/bin/bash
# round 6: the OpenCV-form hole filling on the GPU (tests against oracle/telea_cv.c) + timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inpaint.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_inp6.log 2>&1
rc=$?; echo "inpaint tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/t_inp6.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/inpaint_prof.py 20 c2 2>&1 | grep -v amdgpu > gpurun_out/r06_inpaint_times.txt || exit 1
timeout -k 10 180 python tools/inpaint_prof.py 5 c4 2>&1 | grep -v amdgpu >> gpurun_out/r06_inpaint_times.txt || exit 1
cat gpurun_out/r06_inpaint_times.txt
