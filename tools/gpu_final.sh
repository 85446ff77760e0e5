#!/bin/bash
# end-of-round measurement at the final tree: the driver's exact command, then one bench line per config
# (tools/gpu_configs_bench.sh) - files gpurun_out/<tag>_*
set -o pipefail
T=${TAG:-final}
TAG=$T bash tools/gpu_full.sh || exit 1
bash tools/gpu_configs_bench.sh $T || exit 1
