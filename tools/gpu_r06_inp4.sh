#!/bin/bash
# hole filling after a change: the inpaint GPU tests, the random-map stress under 3 launch policies,
# C2 / C4 timings (default policy) and the per-step stamps at C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inpaint.py tests/test_gpu_post2.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/inp4_tests.txt 2>&1 || { tail -20 gpurun_out/inp4_tests.txt; exit 1; }
tail -1 gpurun_out/inp4_tests.txt
timeout -k 10 600 python -u tools/inpaint_stress.py 6 ${STRESS:-100} > gpurun_out/inp4_stress.txt 2>&1 || { tail -5 gpurun_out/inp4_stress.txt; exit 1; }
tail -1 gpurun_out/inp4_stress.txt
timeout -k 10 300 python -u tools/inpaint_policy.py c2 20 0 > gpurun_out/inp4_times.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/inpaint_policy.py c4 5 0 >> gpurun_out/inp4_times.txt 2>&1 || exit 1
grep config gpurun_out/inp4_times.txt
rm -f gpurun_out/stamps4_c2.txt
DSX_INPAINT_STAMPS=$PWD/gpurun_out/stamps4_c2.txt timeout -k 10 300 python -u tools/inpaint_policy.py c2 2 0 > /dev/null 2>&1 || exit 1
wc -l gpurun_out/stamps4_c2.txt
