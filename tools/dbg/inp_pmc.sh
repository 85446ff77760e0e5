#!/bin/bash
# rocprofv3 kernel stats + two PMC passes of the hole-filling march at C2 (step launches only)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ipmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/dbg/inp_prof1.py c2 30"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $P > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/pmc1 -o run -- $P > $O/pmc1.log 2>&1 || echo pmc1 failed
find $O -name "*.csv" | head
