set -o pipefail
mkdir -p gpurun_out/grid
for c in c1 c3 c5 c2 c4; do
  for adj in 0 -1; do
    DSX_VERBOSE=1 DSX_BLOCKS_PER_CU_ADJ=$adj timeout -k 10 120 python bench.py --config $c --steps 50 --no-cpu-baseline --no-volume-roofline > gpurun_out/grid/${c}_$adj.json 2> gpurun_out/grid/${c}_$adj.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/grid/${c}_$adj.json'));print('$c adj=$adj', d['value'], d['roofline']['kernels_ms'])"
    grep "\[dsx\]" gpurun_out/grid/${c}_$adj.err | sort -u
  done
done
