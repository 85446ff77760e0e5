#!/bin/bash
# round-4 cycle: SSD LR pass from the tile (LDSD) + fused OpenCV LR form + deferred LR + F2 tests,
# A/B of C3 / C4 / C2r against the pre-change build, drop-in figures
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_sgbm_lr.py tests/test_bt.py tests/test_gpu_post2.py tests/test_gpu_host_api.py tests/test_inpaint.py > gpurun_out/r04k_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r04k_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04k_tests.txt | head -20; exit $rc; }
CONFIGS="c3 c2 c2r c4 c1 c5" REPS=2 STEPS=500 bash tools/lib_ab.sh r04k_ab tools/explib/libdsx_base.so || exit 1
timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 > gpurun_out/r04k_dropin.json 2> gpurun_out/r04k_dropin.err || { tail -20 gpurun_out/r04k_dropin.err; exit 1; }
cut -c1-400 gpurun_out/r04k_dropin.json
