# background LK: resident waves resting after each item (VISO_LK_BG_NAP_US)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('kernels_breakdown_chunk') or {}; k=d.get('kernels') or {}
print(f\"{sys.argv[2]:10s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  timed-lk {k.get('lkalign',{}).get('avg_ms',0)*1e3:.1f}  \" + '  '.join(f'{kk} {v[\"avg_ms\"]*1e3:.1f}' for kk, v in b.items()))" $1 $2; }
SMALL="--no-cpu --no-svo --rig-steps 0 --no-init --no-config2 --no-other"
for rep in 1 2; do
for nap in 0 2 5 10; do
  VISO_LK_BG_NAP_US=$nap VISO_LK_BG_STATS=1 timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/nap${nap}_$rep.json 2> $OUT/nap${nap}_$rep.err || { tail -20 $OUT/nap${nap}_$rep.err; exit 1; }
  summ $OUT/nap${nap}_$rep.json nap$nap
  grep "lk-bg" $OUT/nap${nap}_$rep.err | tail -1
done
done
