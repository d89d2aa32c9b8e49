#!/bin/bash
# Round-4 dev: the background LK grid's exposed tail (probe build): the chunk's
# last frame from its first ready sighting to its last item, at chunks of 20
# and 64 frames.
set -o pipefail
OUT=gpurun_out/${1:-r04v}
mkdir -p $OUT
export TMPDIR=/tmp
for b in 20 64; do
  BATCH=$b STEPS=$b VISO_LK_BG_STATS=1 timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe_$b.log 2>&1 || { tail -20 $OUT/probe_$b.log; exit 1; }
  echo "== chunk $b"; grep -i "LK\|launches" $OUT/probe_$b.log
done
