#!/bin/bash
# C4 bench lines at the driver's step counts and at the profiler's (1000 / 500): does the run length
# move the LR pass's kernel time?
set -o pipefail
for s in "20 5" "1000 500" "20 5"; do
  set -- $s
  timeout -k 10 300 python3 bench.py --config c4 --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/r04w_c4_$1.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04w_c4_$1.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$1/$2',d['ms_per_step'],r.get('kernels_ms'),r.get('frac'))"
done
