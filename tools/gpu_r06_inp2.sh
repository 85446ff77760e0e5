#!/bin/bash
# hole filling: the three launch policies at C2 / C4 (tools/inpaint_policy.py), then per-step device
# stamps of the all-persistent policy (DSX_INPAINT_STAMPS)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/inpaint_policy.py c2 10 > gpurun_out/r06_inpaint_policy.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/inpaint_policy.py c4 3 >> gpurun_out/r06_inpaint_policy.txt 2>&1 || exit 1
grep config gpurun_out/r06_inpaint_policy.txt
rm -f gpurun_out/stamps_c2.txt gpurun_out/stamps_c4.txt
DSX_INPAINT_STAMPS=$PWD/gpurun_out/stamps_c2.txt timeout -k 10 300 python -u tools/inpaint_policy.py c2 1 > /dev/null 2>&1 || exit 1
DSX_INPAINT_STAMPS=$PWD/gpurun_out/stamps_c4.txt timeout -k 10 300 python -u tools/inpaint_policy.py c4 1 > /dev/null 2>&1 || exit 1
wc -l gpurun_out/stamps_c*.txt
