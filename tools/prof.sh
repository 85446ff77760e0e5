#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes for one bench config (run on the GPU box).
# usage: tools/prof.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
REPO=$PWD
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $REPO/bench.py --steps ${PSTEPS:-1000} --warmup ${PWARM:-500} --streams 1 --no-cpu-baseline --no-volume-roofline --no-batched --no-e2e --no-parity --no-ref-defaults --no-post --no-dropin --video-frames 0 $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- $BENCH > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed: $pmc"
done
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
find $OUT -name "*.csv" | head -50
