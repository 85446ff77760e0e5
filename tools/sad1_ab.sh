#!/bin/bash
# GPU tests, then C1 (and a D=64 video shape) with the SAD1 layout vs the pair layout (DSX_NO_SAD1=1).
set -o pipefail
mkdir -p gpurun_out/sad1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sad1/gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/sad1/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for rep in 1 2; do
  for v in pair sad1; do
    if [ $v = pair ]; then E="DSX_NO_SAD1=1"; else E="DSX_NO_SAD1=0"; fi
    r=$(env $E timeout -k 5 180 python bench.py --config c1 --steps 1000 --warmup 500 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post 2>gpurun_out/sad1/err_$v.txt) || { echo "FAIL $v"; tail -5 gpurun_out/sad1/err_$v.txt; exit 1; }
    echo "$r" > gpurun_out/sad1/bench_c1_$v.json
    echo "c1 $v $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(d['value'], d['parity']['mismatches'], d['roofline'].get('kernels_ms'), d['roofline'].get('kernel'), 'batch4', d.get('batched',{}).get('value'))")"
  done
done
