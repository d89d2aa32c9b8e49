#!/bin/bash
# Dev: per-kernel instruction counts (SQ_INSTS_VALU / SALU / LDS, SQ_WAVES)
# over a short faithful bench, for the product library and a variant ($2).
set -o pipefail
OUT=gpurun_out/${1:-insts}
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --no-svo --no-other --rig-steps 0 --steps 100 --warmup 20"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $OUT/prod -o run --output-format csv -- $B > $OUT/prod.log 2>&1 || { echo "prod pmc failed"; tail -20 $OUT/prod.log; exit 1; }
if [ -n "$2" ]; then
VISO_LIB=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $OUT/var -o run --output-format csv -- $B > $OUT/var.log 2>&1 || { echo "variant pmc failed"; tail -20 $OUT/var.log; exit 1; }
fi
python tools/pmc_insts.py $OUT/prod ${2:+$OUT/var}
