# grid-size sweep (persistent grid override) per config: bash tools/c1sweep.sh "<configs>" "<grids>"
set -o pipefail
for c in ${1:-c1}; do for g in ${2:-0 2048}; do
  timeout -k 10 120 python bench.py --config $c --steps 1000 --warmup 500 --no-cpu-baseline --no-batched --no-e2e --no-volume-roofline --no-parity --no-ref-defaults --grid-blocks $g > gpurun_out/c1g.json 2>gpurun_out/c1g.err || { tail gpurun_out/c1g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c1g.json'));print('$c grid $g', d['value'], d['ms_per_step'])"
done; done
