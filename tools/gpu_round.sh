#!/bin/bash
# One GPU-box pass: GPU tests, smoke(), default bench line, other configs, rocprofv3 trace + PMC.
# usage: bash tools/gpu_round.sh <tag>      (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-round}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
echo "[gpu_round] tests"
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/gpu_tests.txt 2>&1
rc=$?; tail -5 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
echo "[gpu_round] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
echo "[gpu_round] bench default"
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
for c in ${CONFIGS:-c1 c3 c4 c5}; do
  echo "[gpu_round] bench $c"
  timeout -k 10 300 python bench.py --config $c --steps 300 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
done
echo "[gpu_round] rocprof"
for c in ${PROF_CONFIGS:-c2}; do
  bash tools/prof.sh ${TAG}_$c --config $c || exit 1
  bash tools/prof.sh ${TAG}_${c}_volume --config $c --path volume || exit 1
done
echo "[gpu_round] done"
