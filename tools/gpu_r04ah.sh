#!/bin/bash
# round 4: SAD LR pass with the row's partial keys staged in LDS and sent as atomics on consecutive
# words (DSX_LRCOAL) - parity, WRITE_SIZE per launch (C4, C2r) against the build without it, then A/B
set -o pipefail
mkdir -p gpurun_out/r04ah
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_sgbm_lr.py tests/test_gpu_reference_plumbing.py > gpurun_out/r04ah/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04ah/tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04ah/tests.txt | head -20; exit $rc; }
REPO=$PWD
for c in c4 c2r; do for v in nocoal new; do
  if [ $v = new ]; then L=$REPO/depthestimation_amd/libdsx.so; else L=$REPO/tools/explib/libdsx_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && DSX_LIB=$L timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum --output-format csv -d $REPO/gpurun_out/r04ah/pmc_${c}_$v -o run -- python3 $REPO/bench.py --config $c --steps 200 --warmup 50 --streams 1 --no-cpu-baseline --no-volume-roofline --no-batched --no-e2e --no-parity --no-ref-defaults --no-post --no-dropin > $REPO/gpurun_out/r04ah/pmc_${c}_$v.log 2>&1) || { echo "pmc $c $v failed"; exit 1; }
done; done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04ah/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if "bm2" not in r["Kernel_Name"]: continue
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f.split("/")[2], k, {n: round(sum(v) / len(v), 1) for n, v in d.items()})
PY
CONFIGS="c4 c2r" REPS=3 STEPS=1000 bash tools/lib_ab.sh r04ah_ab tools/explib/libdsx_nocoal.so
