set -o pipefail
mkdir -p gpurun_out/grid
for g in 2560 2816 3072 3328; do
  for c in c2 c4; do
    timeout -k 10 120 python bench.py --config $c --steps 100 --no-cpu-baseline --no-volume-roofline --grid-blocks $g > gpurun_out/grid/$c_$g.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/grid/$c_$g.json'));print('$c $g', d['value'], d['roofline']['kernels_ms'])"
  done
done
