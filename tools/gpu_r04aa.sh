#!/bin/bash
# Round-4 dev A/B: one item per head dequeue in the chunk's last frame (the take1last
# variant) against HEAD's library: the LK / KLT / pipeline / config parity
# tests (the whole GPU suite) on the variant, its background-grid tail probe, then driver-argument
# and default bench lines for both libraries.
set -o pipefail
OUT=gpurun_out/${1:-r04aa}
mkdir -p $OUT
export TMPDIR=/tmp
F=$PWD/viso_amd/libviso_amd_take1last.so
VISO_LIB=$F timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=25 > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
BATCH=20 STEPS=20 timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe_20.log 2>&1 || { tail -20 $OUT/probe_20.log; exit 1; }
grep "LK" $OUT/probe_20.log
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk']
print(f\"{sys.argv[2]:22s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  direct {b['direct']['avg_ms']*1e3:6.2f} us/frame  parity {d['parity_vs_oracle']['max_rel_frobenius'] if d.get('parity_vs_oracle') else '-'}\")" $1 $2; }
for rep in 1 2 3; do
for lib in t1last head; do
  if [ $lib = t1last ]; then export VISO_LIB=$F; else unset VISO_LIB; fi
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-svo --rig-steps 0 > $OUT/${lib}_d$rep.json 2> $OUT/${lib}_d$rep.err || { tail -20 $OUT/${lib}_d$rep.err; exit 1; }
  summ $OUT/${lib}_d$rep.json "$lib-driverargs"
  if [ $rep = 1 ]; then
    timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 > $OUT/${lib}_f$rep.json 2> $OUT/${lib}_f$rep.err || { tail -20 $OUT/${lib}_f$rep.err; exit 1; }
    summ $OUT/${lib}_f$rep.json "$lib-default"
  fi
done
done
