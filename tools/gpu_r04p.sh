# background LK at both sizes (no profiler): the driver-argument line with the
# config-2 (1080p) leg, background on / off
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04p
mkdir -p $OUT
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('kernels_breakdown_chunk') or {}; c=d.get('config2') or {}
print(f\"{sys.argv[2]:8s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  c2-track {c.get('tracking_frames_per_s')}  c2-init {c.get('init_frame_us')}  \" + '  '.join(f'{kk} {v[\"avg_ms\"]*1e3:.1f}' for kk, v in b.items()))" $1 $2; }
SMALL="--no-cpu --no-svo --rig-steps 0 --no-init --no-other"
for rep in 1 2; do
  timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/bg_$rep.json 2> $OUT/bg_$rep.err || { tail -20 $OUT/bg_$rep.err; exit 1; }
  summ $OUT/bg_$rep.json bg
  VISO_LK_BG=0 timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/nobg_$rep.json 2> $OUT/nobg_$rep.err || { tail -20 $OUT/nobg_$rep.err; exit 1; }
  summ $OUT/nobg_$rep.json nobg
done
