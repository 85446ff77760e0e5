#!/bin/bash
# per-step trace of one hole-filling call (DSX_INPAINT_TRACE: state + stream-event time per step)
set -o pipefail
mkdir -p gpurun_out
for c in ${CFGS:-c2}; do
  DSX_INPAINT_TRACE=1 timeout -k 10 120 python tools/inpaint_prof.py 0 $c > gpurun_out/trace_$c.txt 2>&1 || exit 1
  grep -c "^step" gpurun_out/trace_$c.txt
done
