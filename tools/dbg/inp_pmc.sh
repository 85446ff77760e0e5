#!/bin/bash
# PMC passes of the hole-filling march at C2 (step launches only): per-dispatch counters of the last
# fill (dev)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ipmc
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/dbg/inp_prof1.py c2 27"
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU" \
           "TCC_REQ_sum TCC_HIT_sum TCC_EA0_RDREQ_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pmc --output-format csv -d $O/pmc$i -o run -- $P > $O/pmc$i.log 2>&1 || echo "pmc$i failed"
done
cd $GRAFT_REPO_ROOT && python3 tools/dbg/inp_pmc_sum.py $O
