#!/bin/bash
# tools/exit_probe.py modes under rocprofv3 --kernel-trace --stats, one process each (exit codes)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ep
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-torch tiny dsx_load dsx_run inpaint inpaint_keep inpaint_notail_keep}; do
  rm -rf $R/gpurun_out/ep/$m
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ep/$m -o run -- python3 $R/tools/exit_probe.py $m > $R/gpurun_out/ep/$m.log 2>&1
  echo "$m rc=$?"
done
true
