#!/bin/bash
# round 4: volume path (K1 + K2) against the pre-change build - has C4's K2 moved?
set -o pipefail
CONFIGS="c4 c2" REPS=3 STEPS=500 EXTRA="--path volume" bash tools/lib_ab.sh r04s_vol_ab tools/explib/libdsx_base.so
