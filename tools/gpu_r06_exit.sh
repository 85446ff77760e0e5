set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inpaint.py tests/test_telea_heap.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_inp.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t_inp.log
MODES="inpaint inpaint_keep" bash tools/exit_probe.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bprof6 -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/bprof6.log 2>&1; echo "bench-under-rocprofv3 rc=$?"
