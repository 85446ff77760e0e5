#!/bin/bash
# round 4: split the r04k matcher changes - tile-read SSD LR pass (LDSD), per-segment kernarg reload,
# per-segment lane-index rebuild - by variant builds, against the pre-change build
set -o pipefail
mkdir -p gpurun_out
CONFIGS="c3 c2 c2r c4 c1 c5" REPS=2 STEPS=500 bash tools/lib_ab.sh r04l_ab tools/explib/libdsx_base.so tools/explib/libdsx_off.so tools/explib/libdsx_noldsd.so tools/explib/libdsx_noldsd_nolane.so tools/explib/libdsx_noldsd_nokarg.so tools/explib/libdsx_ssdxb.so
