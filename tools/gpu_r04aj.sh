#!/bin/bash
# round 4: staging indices recomputed per load in the one-wave SAD side-0/4 builds too (DSX_T4B=3,
# C2's pass 151 -> 133 VGPRs) against the in-tree build (LR builds only): parity with the variant, then A/B
set -o pipefail
mkdir -p gpurun_out/r04aj
DSX_LIB=$PWD/tools/explib/libdsx_t4all.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r04aj/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04aj/tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04aj/tests.txt | head -20; exit $rc; }
CONFIGS="c2 c1" REPS=3 STEPS=1000 bash tools/lib_ab.sh r04aj_ab tools/explib/libdsx_t4all.so
