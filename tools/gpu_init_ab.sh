# Dev A/B of the initialisation path (bench.py's init_path leg) over
# variant libraries, two repetitions.  usage: gpu_init_ab.sh OUT lib1 lib2 ...
# (an argument lib@VAR=VALUE runs lib with that environment variable set)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
for arg in "$@"; do
  lib=${arg%@*}; ev=""; [ "$arg" != "$lib" ] && ev=${arg#*@}
  n=$(basename $lib .so)${ev:+_${ev//=/}}
  env $ev VISO_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-svo --rig-steps 0 --no-config2 --no-other --no-host-ingest > $OUT/${n}_i$rep.json 2> $OUT/${n}_i$rep.err || { tail -20 $OUT/${n}_i$rep.err; exit 1; }
  python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);i=d['init_path']
print(f\"{sys.argv[2]:22s} init {i['init_frame_us']:.1f}  detect {i['detect_frame_us']:.1f}  frames {i['per_frame_us']}  \" + '  '.join(f'{k} {v[\"avg_us\"]:.1f}x{v[\"launches\"]}' for k, v in i['kernels'].items()))" $OUT/${n}_i$rep.json $n
done
done
