set -o pipefail
O=$PWD/gpurun_out/k2
mkdir -p $O
timeout -k 10 300 python bench.py --config c2 --steps 30 --no-cpu-baseline > $O/c2.json 2>$O/c2.err || exit 1
python -c "import json;d=json.load(open('$O/c2.json'));print(d['roofline_volume'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --path volume --steps 5 --warmup 1 --no-cpu-baseline --no-volume-roofline > $O/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --path volume --steps 5 --warmup 1 --no-cpu-baseline --no-volume-roofline > $O/pmc2.log 2>&1 || echo pmc2 failed
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O
