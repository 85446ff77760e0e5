#!/bin/bash
# round-4 cycle: fused OpenCV LR form + deferred LR check + F2 tests, A/B of the headline configs, drop-in
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_sgbm_lr.py tests/test_bt.py tests/test_gpu_post2.py tests/test_gpu_host_api.py tests/test_inpaint.py > gpurun_out/r04j_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r04j_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 > gpurun_out/r04j_dropin.json 2> gpurun_out/r04j_dropin.err || { tail -20 gpurun_out/r04j_dropin.err; exit 1; }
cat gpurun_out/r04j_dropin.json | cut -c1-80,230-700
CONFIGS="c2 c2r c4" REPS=2 STEPS=1000 bash tools/lib_ab.sh r04j_ab tools/explib/libdsx_base.so
for rep in 1 2; do
for v in new postnt; do
  if [ $v = new ]; then L=$PWD/depthestimation_amd/libdsx.so; else L=$PWD/tools/explib/libdsx_$v.so; fi
  DSX_LIB=$L timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 --frames 400 > gpurun_out/r04j_dropin_$v.json 2>> gpurun_out/r04j_dropin.err || { tail -20 gpurun_out/r04j_dropin.err; exit 1; }
  echo "$v $(python3 -c "import json;[print(d['config'],d['gpu_ms_per_frame'],d['kernels_ms']) for d in map(json.loads,open('gpurun_out/r04j_dropin_$v.json'))]")"
done
done
