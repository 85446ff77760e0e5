#!/bin/bash
# A/B runner on the GPU box: for each "ENV=VAL" variant, bench each config (fused path).
# usage: VARIANTS="DSX_PRIO=0 DSX_PRIO=1" CONFIGS="c2 c4" bash tools/ab.sh [extra bench args]
set -o pipefail
for c in ${CONFIGS:-c2}; do
  for v in ${VARIANTS:-X=0}; do
    r=$(env ${v//+/ } timeout -k 5 120 python bench.py --config $c --steps ${STEPS:-300} --warmup ${WARM:-500} --no-cpu-baseline --no-volume-roofline --no-e2e "$@" 2>/dev/null) || { echo "FAIL $c $v"; exit 1; }
    echo "$c $v $(echo "$r" | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernels_ms'], 'batch4', d.get('batched',{}).get('value'))")"
  done
done
