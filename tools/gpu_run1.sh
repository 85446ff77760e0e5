set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --check > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && cat gpurun_out/bench_c2.json
for c in c1 c3 c4 c5; do timeout -k 10 200 python bench.py --config $c --steps 50 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1; cat gpurun_out/bench_$c.json; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_c2 -o run -- python /root/repo/bench.py --steps 50 --warmup 5 --no-cpu-baseline > /root/repo/gpurun_out/prof_c2.log 2>&1
echo "prof rc=$?"
find /root/repo/gpurun_out/prof_c2 -name "*stats*" | head
