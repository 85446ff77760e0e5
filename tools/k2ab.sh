#!/bin/bash
# K2 (volume WTA) A/B on the GPU box: volume-path parity tests, then the volume leg of the bench
# (K1 + K2 kernel times and HBM fractions) for each config with the row kernel (DSX_K2=0) and the
# flat streaming kernel (DSX_K2=1, default).
# usage: bash tools/k2ab.sh <tag> [configs...]
set -o pipefail
TAG=${1:-k2ab}; shift
O=$PWD/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "volume" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for c in ${@:-c2 c3 c5}; do
  for k2 in 0 1; do
    DSX_K2=$k2 timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 200 --no-cpu-baseline --no-batched --no-e2e \
      --no-ref-defaults --no-parity > $O/bench_${c}_k2$k2.json 2> $O/bench_${c}_k2$k2.err || { tail -20 $O/bench_${c}_k2$k2.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${c}_k2$k2.json'));v=d.get('roofline_volume') or {};print('$c k2=$k2', {k:(x['kernel_ms'],x['frac']) for k,x in v.items() if isinstance(x,dict)})"
  done
done
