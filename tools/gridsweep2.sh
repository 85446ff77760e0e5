for c in c1 c4; do for g in 768 1024 1536 2048 2560 0; do
r=$(timeout -k 5 120 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-volume-roofline --no-e2e --grid-blocks $g 2>/dev/null) || exit 1
echo "$c grid=$g $(echo "$r" | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernels_ms'], 'b4', d.get('batched',{}).get('value'))")"
done; done
