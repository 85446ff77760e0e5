#!/bin/bash
# A/B of inpaint variant libraries (dev): timing at C2 / C4 and the split-parity check
for L in "" tools/dbg/xl/libdsx_ck.so tools/dbg/xl/libdsx_ctv.so tools/dbg/xl/libdsx_both.so; do
  echo "== ${L:-in-tree}"
  if [ -n "$L" ]; then export DSX_LIB=$PWD/$L; else unset DSX_LIB; fi
  timeout -k 10 60 python tools/inpaint_prof.py 20 c2 2>&1 | grep -v amdgpu
  timeout -k 10 60 python tools/inpaint_prof.py 10 c4 2>&1 | grep -v amdgpu
  timeout -k 10 60 python tools/dbg/inp_split.py 2>&1 | grep -v amdgpu | awk '{s+=$5} END {print "split mismatches", s}'
done
