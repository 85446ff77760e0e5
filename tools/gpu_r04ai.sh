#!/bin/bash
# round 4: SAD staging indices recomputed per load in the LR and R >= 6 builds (VGPR spills 36 -> 13 of
# the 312 matcher kernels): parity, then the shapes whose code changed against the committed build
set -o pipefail
mkdir -p gpurun_out/r04ai
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_sgbm_lr.py tests/test_gpu_reference_plumbing.py > gpurun_out/r04ai/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04ai/tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04ai/tests.txt | head -20; exit $rc; }
for rep in 1 2 3; do for v in tools/explib/libdsx_nocoal.so depthestimation_amd/libdsx.so; do
  DSX_LIB=$PWD/$v timeout -k 5 120 python3 tools/shape_time.py --config c1 --checks --num-disp 140 | tee -a gpurun_out/r04ai/shape.txt || exit 1
done; done
CONFIGS="c5 c2r c4" REPS=3 STEPS=500 bash tools/lib_ab.sh r04ai_ab tools/explib/libdsx_nocoal.so
