#!/bin/bash
# round 4: deferred LR check with the key rows staged in LDS (spk_tile) - tests, then the drop-in
# figures with the LDS windows and with the global gathers (DSX_LR_GATHER=1), alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_post2.py tests/test_gpu_host_api.py tests/test_sgbm_lr.py > gpurun_out/r04q_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r04q_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04q_tests.txt | head -20; exit $rc; }
for rep in 1 2; do
  for g in lds gather; do
    if [ $g = gather ]; then export DSX_LR_GATHER=1; else unset DSX_LR_GATHER; fi
    timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 --frames 400 > gpurun_out/r04q_dropin_${g}_$rep.json 2>> gpurun_out/r04q_dropin.err || { tail -20 gpurun_out/r04q_dropin.err; exit 1; }
    echo "$g $(python3 -c "import json;[print(d['config'],d['gpu_ms_per_frame'],d['kernels_ms']) for d in map(json.loads,open('gpurun_out/r04q_dropin_${g}_$rep.json'))]")"
  done
done
