#!/bin/bash
# round 4: matcher with per-segment kernarg reload (LR pass) and the 4-wave SSD lane rebuild (0 B
# scratch), tile-read SSD LR pass off: GPU tests, then every config against the pre-change build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_sgbm_lr.py tests/test_bt.py tests/test_bench_multirank.py tests/test_gpu_post2.py tests/test_gpu_host_api.py > gpurun_out/r04o_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r04o_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04o_tests.txt | head -20; exit $rc; }
CONFIGS="c3 c2 c2r c4 c1 c5" REPS=2 STEPS=500 bash tools/lib_ab.sh r04o_ab tools/explib/libdsx_base.so
