# overlap ubench (two hardware queues / any-order launches hiding the
# dependent-launch gap); parity tests of the product library (direct-pose
# range pre-reduction + rig prologue preload); then the A/Bs: product vs
# no range pre-reduction (driver arguments / default) and product vs no rig
# preload (rig timesteps/s)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 120 ./tools/ubench/overlap_bench > $OUT/overlap.jsonl 2>&1; echo "overlap rc=$?"; cat $OUT/overlap.jsonl
TESTS="tests/test_00_configs.py tests/test_rig_direct.py tests/test_pipeline.py tests/test_golden.py tests/test_track.py tests/test_fast_mode.py" \
  bash tools/gpu_ab3.sh r04g viso_amd/libviso_amd.so viso_amd/libviso_amd_norange.so || exit 1
for lib in viso_amd/libviso_amd.so viso_amd/libviso_amd_norigpre.so; do
  n=$(basename $lib .so)
  VISO_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-svo --no-other --no-init --no-config2 --rig-steps 64 > $OUT/${n}_rig.json 2> $OUT/${n}_rig.err || { tail -20 $OUT/${n}_rig.err; exit 1; }
  python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['rig_direct']
print(sys.argv[2], 'rig faithful', r['faithful']['timesteps_per_s'], 'fast', r['fast']['timesteps_per_s'])" $OUT/${n}_rig.json $n
done
