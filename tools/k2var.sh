#!/bin/bash
# K1/K2 timings of the volume path per config (bench volume leg; VARS repeats the run, exported as DSX_K2_VAR for
# experiment builds that read it)
set -o pipefail
O=$PWD/gpurun_out/${1:-k2var}; shift
mkdir -p $O
for c in ${CONFIGS:-c2 c5}; do
  for v in ${VARS:-0 1}; do
    DSX_K2_VAR=$v timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 200 --no-cpu-baseline --no-batched --no-e2e \
      --no-ref-defaults --no-parity > $O/bench_${c}_v$v.json 2> $O/bench_${c}_v$v.err || { tail -20 $O/bench_${c}_v$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${c}_v$v.json'));v=d.get('roofline_volume') or {};print('$c var=$v', {k:(x['kernel_ms'],x['frac']) for k,x in v.items() if isinstance(x,dict)})"
  done
done
