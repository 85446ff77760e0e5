#!/bin/bash
# round 4: frames in flight in the bench's timed region (--streams 3): bench GPU tests, the driver's
# command, then every config at --streams 3 and --streams 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_multirank.py tests/test_multigpu.py tests/test_gpu_reference_plumbing.py > gpurun_out/r04aa_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r04aa_tests.txt; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 TAG=r04aa bash tools/gpu_full.sh || exit 1
for c in c1 c2 c2r c3 c4 c5; do
  for s in 3 1; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --streams $s --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --no-ref-defaults --no-dropin > gpurun_out/r04aa_${c}_s$s.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r04aa_${c}_s$s.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c s$s',d['value'],d['ms_per_step'],r.get('kernel_ms'),r.get('frac'),d['parity']['mismatches'])"
  done
done
