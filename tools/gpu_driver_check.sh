#!/bin/bash
# GPU tests, then the driver's exact bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5)
# with its wall time, and optional extra configs.  One gpurun call.
# usage: bash tools/gpu_driver_check.sh <tag> [configs...]     (outputs under gpurun_out/<tag>/)
set -o pipefail
O=$PWD/gpurun_out/${1:-check}; shift
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.txt 2>&1
  rc=$?; tail -4 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
fi
t0=$(date +%s.%N)
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || { tail -20 $O/driver_bench.err; exit 1; }
t1=$(date +%s.%N)
python3 -c "print('driver bench wall_s', round($t1 - $t0, 1))" | tee $O/driver_bench.wall
python3 tools/summarize_bench.py $O/driver_bench.json
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --config $c --steps 500 --warmup 200 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python3 tools/summarize_bench.py $O/bench_$c.json
done
