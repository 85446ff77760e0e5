#!/bin/bash
# full GPU cycle: every GPU test, smoke, the driver's exact bench command
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-full}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || tail -4 gpurun_out/${T}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { cat gpurun_out/${T}_smoke.txt; exit 1; }
cat gpurun_out/${T}_smoke.txt
t0=$(date +%s.%N)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver_bench.json 2> gpurun_out/${T}_driver_bench.err || { tail -30 gpurun_out/${T}_driver_bench.err; exit 1; }
python3 -c "import time;print(f'{time.time()-$t0:.1f} s wall')" | tee gpurun_out/${T}_driver_bench.wall
python3 -c "
import json;d=json.load(open('gpurun_out/${T}_driver_bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],'parity',d['parity']['mismatches'])
print('unsettled',d['unsettled'])
print('sharding',d['sharding']['backend'])
for c in ('c2','c4'):
  r=d['dropin'][c]; print('dropin',c,r['value'],r['ms_per_frame'],r['post_processing_ms'],r['kernels_ms'],r['parity']['mismatches'])
print('cpu',d['cpu_baseline']['value'],d['cpu_baseline']['cores'])
"
