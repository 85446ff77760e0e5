#!/bin/bash
# Steady-state shader clock of the fused pass per library: SQ_BUSY_CYCLES (summed over the SEs) and
# GRBM_GUI_ACTIVE per dispatch under rocprofv3 --pmc, with the kernel-trace duration of the same run.
# usage: bash tools/clock_probe.sh <tag> <config> <lib> [lib...]   ("new" = in-tree build)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; C=$2; shift 2
mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/depthestimation_amd/libdsx.so; else L=$GRAFT_REPO_ROOT/$v; fi
  n=$(basename $v .so)
  B="python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 1000 --warmup 500 --no-cpu-baseline --no-volume-roofline --no-batched --no-e2e --no-parity --no-ref-defaults --no-post"
  DSX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n/trace -o run -- $B > $O/$n.trace.log 2>&1 || { echo "trace failed $n"; exit 1; }
  DSX_LIB=$L timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $O/$n/pmc -o run -- $B > $O/$n.pmc.log 2>&1 || { echo "pmc failed $n"; exit 1; }
  python3 - $O/$n <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
st = glob.glob(d + '/trace/**/*kernel_stats.csv', recursive=True)
for r in csv.DictReader(open(st[0])):
    if 'bm2' in r['Name']: print(d.split('/')[-1], 'kernel avg ns', r['AverageNs'], 'calls', r['Calls'])
pc = glob.glob(d + '/pmc/**/*counter_collection.csv', recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(pc[0])):
    if 'bm2' in r['Kernel_Name']: acc[r['Counter_Name']].append(float(r['Counter_Value']))
print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
done
