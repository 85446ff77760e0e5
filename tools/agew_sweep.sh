#!/bin/bash
# Age-level weight sweep (DSX_AGEW, single-frame fused pass): each setting benched per config,
# alternating, REPS times.  usage: CONFIGS="c2 c4" REPS=2 bash tools/agew_sweep.sh <tag> "78,70,64,64" "80,70,62,62" ...
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for c in ${CONFIGS:-c2}; do
  for w in "$@"; do
    r=$(DSX_AGEW=$w timeout -k 5 120 python bench.py --config $c --steps ${STEPS:-1000} --warmup 300 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --no-ref-defaults 2>$O/err.txt) || { echo "FAIL $c $w"; tail -5 $O/err.txt; exit 1; }
    echo "$c $w $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(d['value'], d['parity']['mismatches'], d['roofline'].get('kernels_ms'))")" | tee -a $O/sweep.txt
  done
done
done
