#!/bin/bash
# round 4: the one-stream kernel timing pass of the LR configs at 100 and 500 launches (C4)
set -o pipefail
for rep in 1 2; do for n in 100 500; do
timeout -k 5 200 python3 bench.py --config c4 --steps 20 --warmup 5 --breakdown-steps $n --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --no-ref-defaults --no-dropin 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('c4',$n,d['value'],d['roofline']['kernels_ms'])" || exit 1
done; done
