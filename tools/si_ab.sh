set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_host_api.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/si_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/si_tests.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="X=0 DSX_LIB=$PWD/tools/explib/libdsx_oldinit.so X=0 DSX_LIB=$PWD/tools/explib/libdsx_oldinit.so" CONFIGS="c2 c1 c4 c5" STEPS=1000 bash tools/ab.sh --no-parity --no-batched --no-ref-defaults --no-post
