set -o pipefail
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "volume or sgm" --timeout 120 --timeout-method thread > gpurun_out/k2p_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/k2p_tests.txt; [ $rc -eq 0 ] || exit $rc
PSTEPS=200 PWARM=100 bash tools/prof.sh r02f_c2_volume --config c2 --path volume || exit 1
PSTEPS=100 PWARM=50 bash tools/prof.sh r02f_c3_volume --config c3 --path volume || exit 1
