#!/bin/bash
# round 6: the whole GPU test suite, smoke, and the hole-filling stress (3 launch policies vs the oracle)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r06_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAIL|Error" gpurun_out/r06_gpu_tests.txt | head -20; tail -1 gpurun_out/r06_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.txt 2>&1 || exit 1
tail -1 gpurun_out/r06_smoke.txt
timeout -k 10 600 python -u tools/inpaint_stress.py 6 ${STRESS:-200} > gpurun_out/r06_inpaint_stress.txt 2>&1 || exit 1
tail -2 gpurun_out/r06_inpaint_stress.txt
