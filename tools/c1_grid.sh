#!/bin/bash
# C1 persistent-grid sweep for the SAD1 kernel (bench --grid-blocks), one line per grid size.
set -o pipefail
for g in 0 1024 1536 2048 2560 3072; do
  r=$(DSX_VERBOSE=1 timeout -k 5 120 python bench.py --config c1 --steps 1000 --warmup 500 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --grid-blocks $g 2>/tmp/e_$g.txt) || { echo "FAIL $g"; tail -3 /tmp/e_$g.txt; exit 1; }
  echo "grid $g $(grep -m1 'grid' /tmp/e_$g.txt | cut -c1-90) $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(d['value'], d['parity']['mismatches'], d['roofline'].get('kernels_ms'))")"
done
