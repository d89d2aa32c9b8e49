#!/bin/bash
# Round-4 dev: LK alignment's slowest points (probe build): their GN
# iterations and times, with the background grid and batched after the chain.
set -o pipefail
OUT=gpurun_out/${1:-r04y}
mkdir -p $OUT
export TMPDIR=/tmp
BATCH=20 STEPS=20 timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe_bg.log 2>&1 || { tail -20 $OUT/probe_bg.log; exit 1; }
echo "== background"; grep "LK" $OUT/probe_bg.log
VISO_LK_BG=0 BATCH=20 STEPS=20 timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe_batched.log 2>&1 || { tail -20 $OUT/probe_batched.log; exit 1; }
echo "== batched"; grep "LK" $OUT/probe_batched.log
