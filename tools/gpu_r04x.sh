#!/bin/bash
# round 4: transposed v_sad_u8 segment init for the SAD1 builds - parity, then C1 against the build
# without it (same tree, DSX_SADINIT_ABS=0) and the pre-round base
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_reference_plumbing.py tests/test_sgbm_lr.py > gpurun_out/r04x_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r04x_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04x_tests.txt | head -20; exit $rc; }
CONFIGS="c1" REPS=4 STEPS=1000 bash tools/lib_ab.sh r04x_ab tools/explib/libdsx_nosi1.so || exit 1
