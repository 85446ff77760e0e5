#!/bin/bash
# round 4: host cost per call (one environment pass per launch, cheaper Python checks)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_host_api.py tests/test_gpu_parity.py tests/test_abi.py tests/test_multigpu.py > gpurun_out/r04ae_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04ae_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r04ae_tests.txt | head; exit $rc; }
timeout -k 10 200 python3 tools/host_call_probe.py > gpurun_out/r04ae_host.json 2>/dev/null || exit 1
cat gpurun_out/r04ae_host.json
for c in c1 c2 c4; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --no-ref-defaults --no-dropin > gpurun_out/r04ae_$c.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ae_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['parity']['mismatches'])"
done
