#!/bin/bash
# Hole filling on the GPU box, one parameterised script (round 6).  Runs the named parts in order and
# stops at the first failure; outputs land in gpurun_out/inpaint_*.
#   tests        the hole-filling and post-processing GPU tests (in-tree build)
#   stress       tools/inpaint_stress.py: random maps under 3 launch policies against the oracle (STRESS=N)
#   times        C2 / C4 fill times, default launch policy (tools/inpaint_policy.py)
#   policies     C2 / C4 fill times under the all-persistent and the default policy
#   ab           library A/B of the default policy, alternating: LIBS="tools/varlib/a.so ..." against the in-tree build
#   stamps       per-step device stamps of one steady-state call (DSX_INPAINT_STAMPS), C2 and C4
#   trace        per-step state and time with one launch per step (DSX_INPAINT_TRACE), CFGS (default c2)
# usage: bash tools/gpu_inpaint.sh tests stress times     (LIBS=... bash tools/gpu_inpaint.sh ab)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
for part in "$@"; do
  case $part in
    tests)
      timeout -k 10 300 python -u -m pytest tests/test_inpaint.py tests/test_telea_heap.py tests/test_gpu_post2.py -x -q -m gpu \
        --timeout 120 --timeout-method thread > $O/inpaint_tests.txt 2>&1 || { tail -20 $O/inpaint_tests.txt; exit 1; }
      tail -1 $O/inpaint_tests.txt ;;
    stress)
      timeout -k 10 600 python -u tools/inpaint_stress.py 6 ${STRESS:-100} > $O/inpaint_stress.txt 2>&1 || { tail -5 $O/inpaint_stress.txt; exit 1; }
      tail -1 $O/inpaint_stress.txt ;;
    times|policies)
      P=0; [ $part = policies ] && P=-1,0
      : > $O/inpaint_$part.txt
      for c in c2 c4; do
        n=20; [ $c = c4 ] && n=5
        timeout -k 10 300 python -u tools/inpaint_policy.py $c $n $P >> $O/inpaint_$part.txt 2>&1 || { tail -5 $O/inpaint_$part.txt; exit 1; }
      done
      grep config $O/inpaint_$part.txt ;;
    ab)
      : > $O/inpaint_ab.txt
      for rep in 1 2; do
        for v in $LIBS new; do
          if [ $v = new ]; then L=$GRAFT_REPO_ROOT/depthestimation_amd/libdsx.so; else L=$GRAFT_REPO_ROOT/$v; fi
          DSX_LIB=$L timeout -k 10 300 python -u tools/inpaint_policy.py c2 10 0 >> $O/inpaint_ab.txt 2>&1 || { tail -5 $O/inpaint_ab.txt; exit 1; }
          DSX_LIB=$L timeout -k 10 300 python -u tools/inpaint_policy.py c4 4 0 >> $O/inpaint_ab.txt 2>&1 || { tail -5 $O/inpaint_ab.txt; exit 1; }
        done
      done
      grep config $O/inpaint_ab.txt ;;
    stamps)
      for c in c2 c4; do
        rm -f $O/inpaint_stamps_$c.txt
        DSX_INPAINT_STAMPS=$PWD/$O/inpaint_stamps_$c.txt timeout -k 10 300 python -u tools/inpaint_policy.py $c 1 0 > /dev/null 2>&1 || exit 1
      done
      wc -l $O/inpaint_stamps_c*.txt ;;
    trace)
      for c in ${CFGS:-c2}; do
        DSX_INPAINT_TRACE=1 timeout -k 10 120 python tools/inpaint_prof.py 0 $c > $O/inpaint_trace_$c.txt 2>&1 || exit 1
        grep -c "^step" $O/inpaint_trace_$c.txt
      done ;;
    *) echo "unknown part: $part"; exit 2 ;;
  esac
done
