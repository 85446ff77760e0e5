#!/bin/bash
# round 4: the driver's exact command (20 / 5 steps) with the timed lanes' in_flight handles (auto) and
# without (--in-flight 0), 4 alternating repetitions
set -o pipefail
mkdir -p gpurun_out/r04ao
for rep in 1 2 3 4; do for f in 0 auto; do
  timeout -k 5 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --in-flight $f > gpurun_out/r04ao/b_${f}_$rep.json 2>/dev/null || { echo "FAIL $f"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04ao/b_${f}_$rep.json'));print('$f', d['value'], d['ms_per_step'], d['streams']['in_flight_handles'], d['parity']['mismatches'])" | tee -a gpurun_out/r04ao/ab.txt
done; done
