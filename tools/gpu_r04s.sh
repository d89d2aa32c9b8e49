# background LK: two items per head dequeue (product) vs one (take1): the
# config-1 tests over the LK forms, the drain's share of a chunk, the A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_00_configs.py -k config1 -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/configs.log 2>&1 || { tail -40 $OUT/configs.log; exit 1; }
tail -1 $OUT/configs.log
SMALL="--no-cpu --no-svo --rig-steps 0 --no-init --no-config2 --no-other"
for lib in viso_amd/libviso_amd.so viso_amd/libviso_amd_take1.so; do
  n=$(basename $lib .so)
  VISO_LIB=$PWD/$lib VISO_LK_BG_STATS=1 timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/${n}_d20.json 2> $OUT/${n}_d20.err || { tail -20 $OUT/${n}_d20.err; exit 1; }
  grep "lk-bg" $OUT/${n}_d20.err | tail -2
  VISO_LIB=$PWD/$lib VISO_LK_BG_STATS=1 timeout -k 10 150 python -u bench.py --gpus 1 --steps 64 --warmup 5 $SMALL > $OUT/${n}_d64.json 2> $OUT/${n}_d64.err || { tail -20 $OUT/${n}_d64.err; exit 1; }
  grep "lk-bg" $OUT/${n}_d64.err | tail -2
done
TESTS="tests/test_golden.py" bash tools/gpu_ab3.sh r04s viso_amd/libviso_amd.so viso_amd/libviso_amd_take1.so
