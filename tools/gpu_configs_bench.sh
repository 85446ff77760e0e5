#!/bin/bash
# Final-tree per-config bench lines: bench.py at the driver's step counts for every
# BASELINE config and the C2 shape with the reference defaults, the fused and the volume path; lines land
# in gpurun_out/<tag>_bench_<config>[_volume].json.  usage: bash tools/gpu_configs_bench.sh <tag>
set -o pipefail
T=$1
mkdir -p gpurun_out
for c in c1 c3 c4 c5 c2r; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || { tail -20 gpurun_out/${T}_bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench_$c.json'));r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r.get('frac'),r.get('kernels_ms'),d['parity']['mismatches'])"
done
for c in c2 c4; do
  timeout -k 10 300 python3 bench.py --config $c --path volume --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench_${c}_volume.json 2> gpurun_out/${T}_bench_${c}_volume.err || { tail -20 gpurun_out/${T}_bench_${c}_volume.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench_${c}_volume.json'));r=d['roofline'];print('${c}_volume',d['value'],r.get('frac'),r.get('kernels_ms'),d['parity']['mismatches'])"
done
