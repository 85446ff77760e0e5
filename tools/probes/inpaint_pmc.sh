#!/bin/bash
# Per-step PMC of one steady-state C2 (or $1) hole-filling call: each tl_step dispatch of the last call
# with its counters, two separate --pmc passes (gpurun_out/inpaint_pmc_<config>.txt).  The step order
# matches DSX_INPAINT_STAMPS' (every step is a launch in steady state).
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-c2}
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf $R/gpurun_out/inppmc$i
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/inppmc$i -o run -- python3 $R/tools/inpaint_policy.py $C 1 0 > $R/gpurun_out/inppmc$i.log 2>&1 || { tail -5 $R/gpurun_out/inppmc$i.log; exit 1; }
done
python3 - "$R" "$C" > $R/gpurun_out/inpaint_pmc_$C.txt <<'PY'
import csv, glob, sys
from collections import defaultdict
R, C = sys.argv[1], sys.argv[2]
cols, rows = [], None
for p in (1, 2):
    f = glob.glob(R + "/gpurun_out/inppmc%d/**/*counter_collection.csv" % p, recursive=True)[0]
    d = defaultdict(dict)
    name = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[k] = r["Kernel_Name"]
    ks = sorted(d)
    start = [k for k in ks if "tl_init_a" in name[k]][-1]
    steps = [k for k in ks if k > start and "tl_step" in name[k]]
    cn = sorted(d[steps[0]])
    cols += cn
    vals = [[d[k][c] for c in cn] for k in steps]
    rows = vals if rows is None else [a + b for a, b in zip(rows, vals)]
print("config", C, "steps", len(rows))
print("step " + " ".join(cols))
for s, v in enumerate(rows):
    print(s, " ".join("%.0f" % x for x in v))
PY
rm -rf $R/gpurun_out/inppmc1 $R/gpurun_out/inppmc2
head -3 $R/gpurun_out/inpaint_pmc_$C.txt
