#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes of the drop-in pipeline (tools/dropin_bench.py: StereoCore
# defaults, one dsx_process_pair_device per frame) for one config; reduced into profiles/ by
# tools/make_profiles.py (traffic.json / valu_counts.json keys "<config>:dropin:<kernel>").
# usage: bash tools/gpu_prof_dropin.sh <tag> <config>
set -o pipefail
TAG=$1; C=$2
REPO=$PWD
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python3 $REPO/tools/dropin_bench.py --configs $C --frames 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed: $pmc"
done
cd $REPO
python3 tools/make_profiles.py gpurun_out/prof_$TAG $TAG $C dropin > /dev/null && rm -rf gpurun_out/prof_$TAG
mkdir -p gpurun_out/${TAG}_profiles && cp profiles/${TAG}_* profiles/traffic.json profiles/valu_counts.json gpurun_out/${TAG}_profiles/
