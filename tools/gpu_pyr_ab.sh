#!/bin/bash
# Image-pass A/B (dev): image GPU tests, then per library (product, $2):
# kernel durations of the batched pyramid at 50 and 20 images and FETCH_SIZE /
# WRITE_SIZE passes.  Usage: bash tools/gpu_pyr_ab.sh TAG [variant.so]
set -o pipefail
T=${1:-pyrab}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_image.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in prod ${@:2}; do
  if [ "$lib" != prod ]; then export VISO_LIB=$lib; fi
  tag=$(basename $lib .so)
  for n in ${NS:-50 20}; do
    IMAGES=$n REPS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${tag}_k$n -o run -- python -u tools/bench_pyramid.py > $OUT/${tag}_k$n.log 2>&1 || { tail -20 $OUT/${tag}_k$n.log; exit 1; }
    python tools/db2stats.py $OUT/${tag}_k$n/run_results.db $OUT/${tag}_k$n.csv
    echo "$tag $n images"; grep -E "pyr_" $OUT/${tag}_k$n.csv | cut -c1-200; grep "images/launch" $OUT/${tag}_k$n.log
    IMAGES=$n REPS=5 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/${tag}_f$n -o run --output-format csv -- python -u tools/bench_pyramid.py > $OUT/${tag}_f$n.log 2>&1 || { tail -5 $OUT/${tag}_f$n.log; exit 1; }
    IMAGES=$n REPS=5 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/${tag}_w$n -o run --output-format csv -- python -u tools/bench_pyramid.py > $OUT/${tag}_w$n.log 2>&1 || { tail -5 $OUT/${tag}_w$n.log; exit 1; }
  done
done
echo done
