#!/bin/bash
# rocprofv3 kernel stats + PMC passes for every bench config (fused) and the C2 / C4 volume path,
# reduced on the box by tools/make_profiles.py (raw traces are too large to copy back); the
# summaries land in gpurun_out/<tag>_profiles/.
# usage: bash tools/gpu_prof_round.sh <tag> [configs...]     (VOL="c2 c4" picks the volume-path set,
#        VOL=none skips it; FUSED=none skips the fused set)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/${TAG}_profiles
mkdir -p $OUT
run() {  # tag config path [bench args]
  local t=$1 c=$2 p=$3; shift 3
  echo "[prof] $t $(date +%T)"
  bash tools/prof.sh $t --config $c --path $p "$@" > /dev/null || return 1
  python3 tools/make_profiles.py gpurun_out/prof_$t $t $c $p > /dev/null || return 1
  rm -rf gpurun_out/prof_$t
}
if [ "${FUSED:-}" != none ]; then for c in ${@:-c2 c1 c3 c4 c5 c2r}; do run ${TAG}_$c $c fused || exit 1; done; fi
if [ "${VOL:-}" != none ]; then for c in ${VOL:-c2 c4}; do run ${TAG}_${c}_volume $c volume || exit 1; done; fi
cp profiles/${TAG}_* profiles/traffic.json profiles/valu_counts.json $OUT/
echo "[prof] done $(date +%T)"
