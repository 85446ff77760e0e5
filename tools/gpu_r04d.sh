#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_post2.py tests/test_inpaint.py tests/test_gpu_host_api.py tests/test_bench_multirank.py > gpurun_out/r04d_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r04d_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 tools/post_timeline.py c4 c2r > gpurun_out/r04d_post_tl.json 2>&1 || { tail gpurun_out/r04d_post_tl.json; exit 1; }
cat gpurun_out/r04d_post_tl.json
timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 > gpurun_out/r04d_dropin.json 2> gpurun_out/r04d_dropin.err || { tail -20 gpurun_out/r04d_dropin.err; exit 1; }
cat gpurun_out/r04d_dropin.json
