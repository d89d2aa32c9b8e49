#!/bin/bash
# Dev: LK alignment per-point timing (probe build): slowest point, iteration
# counts, at ingest chunks of 20 and 64 frames.
set -o pipefail
OUT=gpurun_out/${1:-lkprobe}
mkdir -p $OUT
export TMPDIR=/tmp
for b in 20 64; do
  BATCH=$b STEPS=128 timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe_$b.log 2>&1 || { tail -20 $OUT/probe_$b.log; exit 1; }
  echo "== batch $b"; grep "LK alignment" $OUT/probe_$b.log
done
