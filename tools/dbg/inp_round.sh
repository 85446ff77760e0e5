#!/bin/bash
# hole-filling check + timing + kernel trace (dev)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_inpaint.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tinp.log 2>&1 || { tail -30 gpurun_out/tinp.log; exit 1; }
tail -1 gpurun_out/tinp.log
timeout -k 10 60 python tools/inpaint_prof.py 20 c2 2>&1 | grep -v amdgpu
timeout -k 10 60 python tools/inpaint_prof.py 20 c4 2>&1 | grep -v amdgpu
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -- python tools/dbg/inp_prof1.py ${2:-c2} ${1:-26} > gpurun_out/kt.log 2>&1 && python tools/dbg/inp_seq.py gpurun_out/kt
