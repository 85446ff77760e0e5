#!/bin/bash
# round-5 evidence beside tools/gpu_final.sh: hole-filling timings, per-step kernel trace and PMC at
# C2 / C4, the drop-in pipeline, and a rocprofv3 kernel-stats pass of the driver's bench command;
# files gpurun_out/r05x_*
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 120 python tools/inpaint_prof.py 20 c2 2>&1 | grep -v amdgpu > $O/r05x_inpaint_times.txt || exit 1
timeout -k 10 120 python tools/inpaint_prof.py 20 c4 2>&1 | grep -v amdgpu >> $O/r05x_inpaint_times.txt || exit 1
cat $O/r05x_inpaint_times.txt
timeout -k 10 200 python tools/dropin_bench.py --configs c2r c4 --frames 200 2>&1 | grep -v amdgpu > $O/r05x_dropin.json || exit 1
cat $O/r05x_dropin.json | cut -c 1-300
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in c2 c4; do
  st=$([ $c = c2 ] && echo 27 || echo 3000)
  rm -rf $R/$O/kt_$c
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt_$c -- python3 $R/tools/dbg/inp_prof1.py $c $st > $R/$O/kt_$c.log 2>&1 || exit 1
  python3 $R/tools/dbg/inp_seq.py $R/$O/kt_$c > $R/$O/r05x_inpaint_${c}_steps.txt || exit 1
  tail -1 $R/$O/r05x_inpaint_${c}_steps.txt
  rm -rf $R/$O/kt_$c
done
cd $R && bash tools/dbg/inp_pmc.sh > $O/r05x_inpaint_c2_pmc.txt 2>&1 || exit 1
rm -rf $O/ipmc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/bprof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/$O/bprof.log 2>&1 || { tail -20 $R/$O/bprof.log; exit 1; }
cd $R && f=$(find $O/bprof -name "*kernel_stats.csv" | head -1) && cp $f $O/r05x_bench_kernel_stats.csv && rm -rf $O/bprof && head -12 $O/r05x_bench_kernel_stats.csv | cut -c 1-160
