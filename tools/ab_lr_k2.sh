#!/bin/bash
# GPU parity for the LR / volume paths, then old (exp/libdsx_e0.so) vs new (in-tree) timings:
# fused LR pass (tools/lr_cost.py, C2 and C4 shapes) and the volume path's K2 with LR (C4, C3).
# usage: bash tools/ab_lr_k2.sh <tag>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_multigpu.py tests/test_gpu_reference_plumbing.py tests/test_sgbm_lr.py tests/test_bt.py tests/test_sgm.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
OLD=$GRAFT_REPO_ROOT/depthestimation_amd/exp/libdsx_e0.so
for rep in 1 2; do
  for v in new old; do
    L=$GRAFT_REPO_ROOT/depthestimation_amd/libdsx.so; [ $v = old ] && L=$OLD
    for c in c2 c4; do echo "$v lr_cost $(DSX_LIB=$L timeout -k 5 120 python3 tools/lr_cost.py --config $c --iters 300)" | tee -a $O/ab.txt || exit 1; done
    for c in c4 c3; do
      DSX_LIB=$L timeout -k 5 200 python3 bench.py --config $c --path volume --steps 200 --warmup 100 --no-cpu-baseline --no-e2e --no-post --no-batched --no-volume-roofline > $O/vol_${c}_$v.json 2>$O/vol_${c}_$v.err || { tail -5 $O/vol_${c}_$v.err; exit 1; }
      echo "$v volume $c $(python3 -c "import json;d=json.loads(open('$O/vol_${c}_$v.json').read().splitlines()[-1]);print(d['value'], d['roofline']['kernels_ms'], d['parity']['mismatches'])")" | tee -a $O/ab.txt
    done
  done
done
