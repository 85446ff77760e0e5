#!/bin/bash
# rocprofv3 kernel stats + PMC passes (tools/prof.sh) for every bench config, fused path.
# usage: bash tools/gpu_prof_all.sh <tag> [configs...]
set -o pipefail
TAG=$1; shift
for c in ${@:-c1 c2 c3 c4 c5 c2r}; do
  echo "[prof_all] $c"
  bash tools/prof.sh ${TAG}_$c --config $c || exit 1
done
echo "[prof_all] done"
