#!/bin/bash
# C1 single-frame kernel time against blocks per CU (dev)
for adj in 0 -2 -4 -6 -8 -9; do
  r=$(DSX_BLOCKS_PER_CU_ADJ=$adj timeout -k 10 120 python3 bench.py --config c1 --steps 200 --warmup 20 --no-cpu-baseline --streams 1 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'].get('kernels_ms'), d['parity']['mismatches'])")
  echo "adj $adj: $r"
done
