# background LK alignment, robust form (grid launched behind the chunk's first
# direct launches; idle waves leave; errors reported): the whole GPU suite,
# the driver-argument line on / off, and the bench under rocprofv3
# --kernel-trace --stats (no lk_item_kernel may approach the 200 ms bound)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread --durations=25 -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('kernels_breakdown_chunk') or {}; k=d.get('kernels') or {}
print(f\"{sys.argv[2]:14s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  timed-lk {k.get('lkalign',{}).get('avg_ms',0)*1e3:.1f}  \" + '  '.join(f'{kk} {v[\"avg_ms\"]*1e3:.1f}' for kk, v in b.items()))" $1 $2; }
SMALL="--no-cpu --no-svo --rig-steps 0 --no-init --no-config2 --no-other"
for rep in 1 2; do
  timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/bg_$rep.json 2> $OUT/bg_$rep.err || { tail -20 $OUT/bg_$rep.err; exit 1; }
  summ $OUT/bg_$rep.json bg
  VISO_LK_BG=0 timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/nobg_$rep.json 2> $OUT/nobg_$rep.err || { tail -20 $OUT/nobg_$rep.err; exit 1; }
  summ $OUT/nobg_$rep.json nobg
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err; exit 1; }
summ $OUT/bench_prof.json prof
