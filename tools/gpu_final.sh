#!/bin/bash
# end-of-round measurement at the final tree: the driver's exact command, then one bench line per config
# (tools/gpu_configs_bench.sh) - files gpurun_out/<tag>_*.  PROF=1 also runs the driver's command under
# rocprofv3 --kernel-trace --stats (its exit status is the call's; <tag>_bench_kernel_stats.csv).
set -o pipefail
T=${TAG:-final}
TAG=$T bash tools/gpu_full.sh || exit 1
bash tools/gpu_configs_bench.sh $T || exit 1
if [ -n "$PROF" ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/${T}_prof.log 2>&1
  rc=$?; echo "rocprofv3 bench rc=$rc" | tee -a $R/gpurun_out/${T}_prof.log
  cp $(find $R/gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1) $R/gpurun_out/${T}_bench_kernel_stats.csv
  rm -rf $R/gpurun_out/${T}_prof
  exit $rc
fi
