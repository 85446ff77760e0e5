#!/bin/bash
# LR-check configs (C3, C4, C2 with reference defaults): GPU LR parity tests, then fused-pass and
# lr_fixup kernel times.   usage: bash tools/lrab.sh <tag>
set -o pipefail
O=$PWD/gpurun_out/${1:-lrab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c3 c4 c2r}; do
  timeout -k 10 200 python bench.py --config $c --steps 500 --warmup 500 --no-cpu-baseline --no-batched --no-e2e --no-ref-defaults \
    --no-volume-roofline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['roofline']['kernels_ms'], d['parity']['mismatches'])"
done
