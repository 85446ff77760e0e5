#!/bin/bash
# round 4: the bench's timed lanes with in_flight handles (--in-flight 1) against lone-frame handles
# (--in-flight 0), 3 streams, 1000 steps, alternating; every fused config
set -o pipefail
mkdir -p gpurun_out/r04an
for rep in 1 2; do for c in c2 c4 c2r c3 c1 c5; do for f in 0 1; do
  r=$(timeout -k 5 180 python3 bench.py --config $c --steps 1000 --warmup 300 --in-flight $f --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --no-ref-defaults --no-dropin 2>gpurun_out/r04an/err_$c.txt) || { echo "FAIL $c $f"; tail -5 gpurun_out/r04an/err_$c.txt; exit 1; }
  echo "$c in_flight=$f $(echo "$r" | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(d['value'], d['parity']['mismatches'], d['streams']['in_flight_handles'], d['roofline']['kernels_ms'])")" | tee -a gpurun_out/r04an/ab.txt
done; done; done
