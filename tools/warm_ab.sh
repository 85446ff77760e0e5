#!/bin/bash
# C2 headline per-step time against the warm-up: the driver's 20/5 with and without the untimed
# clock-settling phase (--settle seconds), and the long default run.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
F="--no-cpu-baseline --no-batched --no-e2e --no-post --no-ref-defaults --no-volume-roofline"
for rep in 1 2; do
  for sw in "20 5 0" "20 5 0.4" "20 5 1.0" "1000 500 0"; do
    set -- $sw
    echo "steps=$1 warmup=$2 settle=$3 $(timeout -k 5 120 python3 bench.py --steps $1 --warmup $2 --settle $3 $F | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["settle"]["steps"])')" | tee -a $O/warm.txt || exit 1
  done
done
