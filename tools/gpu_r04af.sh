#!/bin/bash
# round 4: the balance knobs (priority bands, age weights) under frames in flight - the next frame now
# fills the tail they were tuned against.  Two repetitions, C2 and C4, 1000 timed steps.
set -o pipefail
for rep in 1 2; do
  VARIANTS="X=0 DSX_PRIO=0 DSX_AGEW=64,64,64,64 DSX_PRIO=0+DSX_AGEW=64,64,64,64" CONFIGS="c2 c4" STEPS=1000 bash tools/ab.sh --no-post --no-batched --no-ref-defaults --no-dropin --no-parity || exit 1
done
