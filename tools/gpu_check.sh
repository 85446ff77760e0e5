#!/bin/bash
# All GPU tests, then the default bench line (and optional extra configs): one gpurun call.
# usage: bash tools/gpu_check.sh <tag> [configs...]
set -o pipefail
O=$PWD/gpurun_out/${1:-check}; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -4 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['ms_per_step'], d['parity']['mismatches'], d.get('e2e_host'))"
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps 500 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['parity']['mismatches'], d.get('e2e_host'))"
done
