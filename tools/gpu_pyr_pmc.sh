#!/bin/bash
# HBM traffic of the image pass (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one
# counter per run) at the default chunk (50 images) and the driver's (20);
# summarise with tools/pmc_traffic.py.  Usage: bash tools/gpu_pyr_pmc.sh TAG
set -o pipefail
TAG=${1:-pyrpmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "50 --steps 100 --warmup 20" "20 --batch 20 --steps 20 --warmup 5"; do
  set -- $cfg; n=$1; shift
  B="python -u bench.py --no-cpu --no-svo --no-other --rig-steps 0 $@"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pyr_f$n -o run --output-format csv -- $B > $OUT/pyr_f$n.log 2>&1 || { echo "pyr_f$n failed"; tail -20 $OUT/pyr_f$n.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pyr_w$n -o run --output-format csv -- $B > $OUT/pyr_w$n.log 2>&1 || { echo "pyr_w$n failed"; tail -20 $OUT/pyr_w$n.log; exit 1; }
  echo pyr $n ok
done
