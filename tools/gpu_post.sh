#!/bin/bash
# F2 cycle on the GPU box: the post-processing / hole-filling / host-API GPU tests, the per-block phase
# timeline of spk_tile + post_tail3 (tools/post_timeline.py) and the drop-in figures (tools/dropin_bench.py).
# usage: TAG=<tag> bash tools/gpu_post.sh
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-post}
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_post2.py tests/test_inpaint.py tests/test_gpu_host_api.py > gpurun_out/${T}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 tools/post_timeline.py c4 c2r > gpurun_out/${T}_post_tl.json 2>&1 || { tail gpurun_out/${T}_post_tl.json; exit 1; }
cat gpurun_out/${T}_post_tl.json
timeout -k 10 300 python3 tools/dropin_bench.py --configs c2r c4 > gpurun_out/${T}_dropin.json 2> gpurun_out/${T}_dropin.err || { tail -20 gpurun_out/${T}_dropin.err; exit 1; }
cat gpurun_out/${T}_dropin.json
