# Dev A/B over several variant libraries: driver-argument and default bench
# lines (no CPU legs) per library, two repetitions, plus the parity tests
# for the product library first.  usage: gpu_ab3.sh OUT lib1 lib2 ...
# (an argument lib@VAR=VALUE runs lib with that environment variable set)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_00_configs.py tests/test_pipeline.py tests/test_golden.py tests/test_geometry.py tests/test_track.py tests/test_stereo_init.py} -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('kernels_breakdown_chunk') or {}; k=d.get('kernels') or {}
print(f\"{sys.argv[2]:26s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  timed-lk {k.get('lkalign',{}).get('avg_ms',0)*1e3:.1f}  \" + '  '.join(f'{kk} {v[\"avg_ms\"]*1e3:.1f}' for kk, v in b.items()))" $1 $2; }
SMALL="--no-cpu --no-svo --rig-steps 0 --no-init --no-config2 --no-other"
for rep in $(seq ${REPS:-2}); do
for arg in "$@"; do
  lib=${arg%@*}; ev=""; [ "$arg" != "$lib" ] && ev=${arg#*@}
  n=$(basename $lib .so)${ev:+_${ev//=/}}
  env $ev VISO_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/${n}_d$rep.json 2> $OUT/${n}_d$rep.err || { tail -20 $OUT/${n}_d$rep.err; exit 1; }
  summ $OUT/${n}_d$rep.json "$n-driver"
  env $ev VISO_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py $SMALL > $OUT/${n}_f$rep.json 2> $OUT/${n}_f$rep.err || { tail -20 $OUT/${n}_f$rep.err; exit 1; }
  summ $OUT/${n}_f$rep.json "$n-default"
done
done
