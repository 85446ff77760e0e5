#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), then the driver's exact bench command (wall time kept).
# usage: bash tools/gpu_final_check.sh <tag>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
t0=$(date +%s.%N)
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_bench.json 2> $O/driver_bench.err || { tail -20 $O/driver_bench.err; exit 1; }
t1=$(date +%s.%N)
python3 -c "print('driver bench wall_s', round($t1 - $t0, 1))" | tee $O/driver_bench.wall
python3 tools/summarize_bench.py $O/driver_bench.json
