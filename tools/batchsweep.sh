set -o pipefail
mkdir -p gpurun_out/batch
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for c in c1 c4 c2; do
  for b in 1 4 8; do
    timeout -k 10 180 python bench.py --config $c --steps 40 --warmup 5 --batch $b --no-cpu-baseline --no-volume-roofline > gpurun_out/batch/${c}_$b.json 2>gpurun_out/batch/${c}_$b.err || { tail -5 gpurun_out/batch/${c}_$b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/batch/${c}_$b.json'));print('$c batch $b', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
  done
done
