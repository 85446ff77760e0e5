#!/bin/bash
# SGM aggregation: GPU tests, then the C2 shape through each mode
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sgm.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sgm_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/sgm_tests.txt; [ $rc -eq 0 ] || exit $rc
for m in ${MODES:-sgbm_3way hh}; do
  timeout -k 10 300 python bench.py --config c2 --sgm $m --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/sgm_$m.json 2> gpurun_out/sgm_$m.err || { tail -20 gpurun_out/sgm_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sgm_$m.json'));print('$m', d['value'], d['ms_per_step'], d['roofline'].get('kernels_ms'), d.get('parity',{}).get('mismatches'))"
done
