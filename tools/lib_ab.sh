#!/bin/bash
# Same-box A/B of libdsx builds: optional GPU tests with the in-tree lib (TESTS="files..."), then
# each config benched with every library, alternating, REPS times.  The first argument after the
# tag is the baseline; "new" stands for the in-tree build.
# usage: CONFIGS="c2r c4 c3" REPS=2 TESTS=tests EXTRA="--path volume" bash tools/lib_ab.sh <tag> <lib> [lib...]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
LIBS="$* new"
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
  rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq ${REPS:-2}); do
for c in ${CONFIGS:-c2r c4 c3}; do
  for v in $LIBS; do
    if [ $v = new ]; then L=$GRAFT_REPO_ROOT/depthestimation_amd/libdsx.so; else L=$GRAFT_REPO_ROOT/$v; fi
    n=$(basename $v .so)
    r=$(DSX_LIB=$L timeout -k 5 180 python bench.py --config $c --steps ${STEPS:-500} --warmup 300 --no-cpu-baseline --no-volume-roofline --no-e2e --no-post --no-batched --no-ref-defaults --no-dropin $EXTRA 2>$O/err_${c}_$n.txt) || { echo "FAIL $c $v"; tail -5 $O/err_${c}_$n.txt; exit 1; }
    echo "$c $n $(echo "$r" | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(d['value'], d['parity']['mismatches'], d['roofline'].get('kernels_ms'))")" | tee -a $O/ab.txt
  done
done
done
