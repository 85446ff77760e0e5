#!/bin/bash
# quick GPU cycle: all GPU tests then the bench configs (fused line + volume roofline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.txt 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { cat gpurun_out/bench_$c.err | tail -20; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));v=d.get('roofline_volume') or {};print('$c', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'], {k:(x['kernel_ms'],x['frac']) for k,x in v.items() if isinstance(x,dict)})"
done
