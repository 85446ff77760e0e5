#!/bin/bash
# round 4: rocprofv3 stats + PMC of the LR passes whose build changed (C4, C2r), one stream; summarised
# on the box (tools/make_profiles.py) and only the summaries kept under gpurun_out/r04ak_out
set -o pipefail
PSTEPS=300 PWARM=100 bash tools/prof.sh r04ak_c4 --config c4 > /dev/null || exit 1
PSTEPS=300 PWARM=100 bash tools/prof.sh r04ak_c2r --config c2r > /dev/null || exit 1
python3 tools/make_profiles.py gpurun_out/prof_r04ak_c4 r04ak_c4 c4 fused || exit 1
python3 tools/make_profiles.py gpurun_out/prof_r04ak_c2r r04ak_c2r c2r fused || exit 1
mkdir -p gpurun_out/r04ak_out
cp profiles/r04ak_* profiles/traffic.json profiles/valu_counts.json gpurun_out/r04ak_out/
rm -rf gpurun_out/prof_r04ak_*
ls gpurun_out/r04ak_out
