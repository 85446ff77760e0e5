#!/bin/bash
# round 4: in-flight handles - pipeline / ABI / stub tests, then the drop-in figures (bench secondary)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multigpu.py tests/test_gpu_reference_plumbing.py tests/test_abi.py tests/test_integration_stub.py tests/test_gpu_host_api.py > gpurun_out/r04ag_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r04ag_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r04ag_tests.txt | head; exit $rc; }
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04ag_bench.json 2>/dev/null || exit 1
python3 -c "
import json;d=json.loads(open('gpurun_out/r04ag_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['parity']['mismatches'])
for c in ('c2','c4'): print(c, d['dropin'][c]['ms_per_frame'], d['dropin'][c]['frames_in_flight_3'])
"
