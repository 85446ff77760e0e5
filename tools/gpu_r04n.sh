#!/bin/bash
# round 4: is the plain left pass (C2 headline) slower because of the OpenCV-form LR key code in SIDE 0?
set -o pipefail
CONFIGS="c2 c1 c5" REPS=4 STEPS=500 bash tools/lib_ab.sh r04n_ab tools/explib/libdsx_base.so tools/explib/libdsx_nosg.so
