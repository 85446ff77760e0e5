#!/bin/bash
# GPU tests with the in-tree lib, then old/new A/B of the LR configs (C3, C4, C2 with reference defaults).
# usage: bash tools/lr_ab.sh <old lib path>
set -o pipefail
OLD=$1
mkdir -p gpurun_out/lrab
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lrab/gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/lrab/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for c in c3 c4 c2; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=$PWD/depthestimation_amd/libdsx.so; fi
    r=$(DSX_LIB=$L timeout -k 5 180 python bench.py --config $c --steps 500 --warmup 500 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched 2>gpurun_out/lrab/err_${c}_${v}.txt) || { echo "FAIL $c $v"; tail -5 gpurun_out/lrab/err_${c}_${v}.txt; exit 1; }
    echo "$c $v $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);rd=d.get('c2_reference_defaults') or {};print(d['value'], d['parity']['mismatches'], d['roofline'].get('kernels_ms'), 'refdef', rd.get('value'), rd.get('kernels_ms'))")"
  done
done
done
