#!/bin/bash
# The drop-in pipeline (StereoCore defaults, estimate_depth_device) on the GPU box: stream-event
# figures, then a rocprofv3 kernel trace + stats of the same script (per-kernel breakdown and the
# gaps between dependent launches).  usage: tools/gpu_dropin.sh <tag> [configs...]
set -o pipefail
TAG=$1; shift
CFGS=${@:-c2r c4}
REPO=$PWD
OUT=$PWD/gpurun_out/dropin_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 tools/dropin_bench.py --configs $CFGS > $OUT/dropin.json 2> $OUT/dropin.err || { tail -20 $OUT/dropin.err; exit 1; }
cat $OUT/dropin.json
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$c -o run -- python3 $REPO/tools/dropin_bench.py --configs $c --frames 50 > $OUT/trace_$c.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace_$c.log; exit 1; }
done
find $OUT -name "*.csv"
