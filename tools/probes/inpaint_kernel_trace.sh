#!/bin/bash
# rocprofv3 kernel trace of repeated C2 fills (tools/inpaint_policy.py), reduced to the last call's
# kernels: init kernels, step count and step-time sum (gpurun_out/inpaint_kernel_trace.txt)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/inpprof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/inpprof -o run -- python3 $R/tools/inpaint_policy.py ${1:-c2} 5 0 > $R/gpurun_out/inpprof.log 2>&1 || exit 1
python3 - "$R" > $R/gpurun_out/inpaint_kernel_trace.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/gpurun_out/inpprof/**/*kernel_trace.csv", recursive=True)[0]
seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48]) for r in csv.DictReader(open(f)))
i = [k for k, (a, b, n) in enumerate(seq) if "tl_init_a" in n][-1]
last = seq[i:]
t0 = last[0][0]
for a, b, n in last[:3]:
    print(n, "start_us %.1f" % ((a - t0) / 1e3), "dur_us %.1f" % ((b - a) / 1e3))
d = [(b - a) / 1e3 for a, b, n in last if "tl_step" in n]
print("steps", len(d), "sum_us %.1f" % sum(d), "median_us %.1f" % sorted(d)[len(d) // 2], "span_us %.1f" % ((last[-1][1] - t0) / 1e3))
PY
rm -rf $R/gpurun_out/inpprof
cat $R/gpurun_out/inpaint_kernel_trace.txt
