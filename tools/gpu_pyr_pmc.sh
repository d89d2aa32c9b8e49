#!/bin/bash
# HBM traffic of the image pass (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one
# counter per run) over bench.py itself, at the chunks its lines time: the
# driver's arguments (one 20-image chunk: the tail launch also copies the
# chunk's last level 0 and clears the background-LK words) and the default
# line's tracking chunks (64 images: background-LK chunks are cut to
# kLkBatch); summarised by tools/pmc_traffic.py into $OUT/pyramid_traffic.json,
# each entry stamped with the loaded library's source hash (bench.py ignores
# an entry whose hash is not the library's).  Usage: bash tools/gpu_pyr_pmc.sh TAG
set -o pipefail
TAG=${1:-pyrpmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SRC=$(timeout -k 10 60 python -c "import viso_amd._lib as l; print(l.built_hash())") || { echo "library hash failed"; exit 1; }
SMALL="--no-cpu --no-svo --no-other --rig-steps 0 --no-init --no-config2 --no-host-ingest"
for cfg in "20 --batch 20 --steps 20 --warmup 5" "64 --steps 128 --warmup 20"; do
  set -- $cfg; n=$1; shift
  B="python -u bench.py $SMALL $@"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pyr_f$n -o run --output-format csv -- $B > $OUT/pyr_f$n.log 2>&1 || { echo "pyr_f$n failed"; tail -20 $OUT/pyr_f$n.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pyr_w$n -o run --output-format csv -- $B > $OUT/pyr_w$n.log 2>&1 || { echo "pyr_w$n failed"; tail -20 $OUT/pyr_w$n.log; exit 1; }
  F=$(find $OUT/pyr_f$n -name '*counter_collection.csv' | head -1); W=$(find $OUT/pyr_w$n -name '*counter_collection.csv' | head -1)
  IMAGES=$n SRC_HASH=$SRC SOURCE="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over bench.py $* (tools/gpu_pyr_pmc.sh $TAG)" \
    python tools/pmc_traffic.py $(dirname $F) $(dirname $W) $OUT/pyramid_traffic.json > $OUT/pyr_traffic_$n.log || { echo "pmc_traffic $n failed"; exit 1; }
  echo pyr $n ok
done
