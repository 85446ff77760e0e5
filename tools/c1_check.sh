#!/bin/bash
# GPU tests + C1 line (default grid) after a launch-geometry change.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c1check_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/c1check_tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 5 180 python bench.py --config c1 --steps 1000 --warmup 500 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post > gpurun_out/c1check_bench_$rep.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c1check_bench_$rep.json').read().strip().splitlines()[-1]);print('c1', d['value'], d['parity']['mismatches'], d['roofline'].get('kernels_ms'), d['roofline'].get('frac'), 'batch4', d.get('batched',{}).get('value'))"
done
