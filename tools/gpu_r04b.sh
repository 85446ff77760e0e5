#!/bin/bash
# round 4, first GPU cycle: new F2 / process_pair / inpaint tests, then the drop-in figures
# (new vs legacy F2) and a kernel trace of the drop-in pipeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_post2.py tests/test_inpaint.py tests/test_gpu_host_api.py > gpurun_out/r04b_tests.txt 2>&1
rc=$?; tail -25 gpurun_out/r04b_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 > gpurun_out/r04b_dropin.json 2> gpurun_out/r04b_dropin.err || { tail -20 gpurun_out/r04b_dropin.err; exit 1; }
timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 --legacy-post > gpurun_out/r04b_dropin_legacy.json 2>> gpurun_out/r04b_dropin.err || { tail -20 gpurun_out/r04b_dropin.err; exit 1; }
cat gpurun_out/r04b_dropin.json gpurun_out/r04b_dropin_legacy.json
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
for c in c2r c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/r04b_trace_$c -o run -- python3 $REPO/tools/dropin_bench.py --configs $c --frames 50 > $REPO/gpurun_out/r04b_trace_$c.log 2>&1 || { echo "trace failed"; tail -20 $REPO/gpurun_out/r04b_trace_$c.log; exit 1; }
done
find $REPO/gpurun_out/r04b_trace_* -name "*stats*"
