#!/bin/bash
# round 6, final tree: every GPU test, smoke, the driver's exact command, one line per config
# (tools/gpu_final.sh), then the driver's command under rocprofv3 --kernel-trace --stats (exit status kept)
set -o pipefail
TAG=${TAG:-r06_final} bash tools/gpu_final.sh || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_final_prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r06_final_prof.log 2>&1
rc=$?; echo "rocprofv3 bench rc=$rc" | tee -a $R/gpurun_out/r06_final_prof.log
cp $(find $R/gpurun_out/r06_final_prof -name "*kernel_stats.csv" | head -1) $R/gpurun_out/r06_final_bench_kernel_stats.csv
rm -rf $R/gpurun_out/r06_final_prof
exit $rc
