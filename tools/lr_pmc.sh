#!/bin/bash
# One PMC pass (8 SQ counters) over the fused pass of each config: VALU/LDS/VMEM instruction counts and
# wave cycles per launch, to split what the LR variant adds.  usage: bash tools/lr_pmc.sh c2 c2r c4
set -o pipefail
REPO=$PWD
mkdir -p gpurun_out/lrpmc
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $REPO/gpurun_out/lrpmc/$c -o run -- python3 $REPO/bench.py --config $c --steps 200 --warmup 50 --no-cpu-baseline --no-volume-roofline --no-batched --no-e2e --no-parity --no-ref-defaults --no-post > $REPO/gpurun_out/lrpmc/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $REPO/gpurun_out/lrpmc/$c.log; exit 1; }
done
cd $REPO && python3 - "$@" <<'PY'
import csv, glob, sys, collections
for c in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/lrpmc/{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "bm2" not in k and "lr_fixup" not in k: continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(c, k[:60], {n: round(sum(v) / len(v) / 1e6, 3) for n, v in sorted(d.items())}, "(M per launch)")
PY
