#!/bin/bash
# Dev A/B: LK alignment launch order (product) against a base library ($2):
# LK / pipeline parity tests, then bench lines at the default and at the
# driver's arguments for both libraries.
set -o pipefail
OUT=gpurun_out/${1:-lkord}
B=$2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_track.py tests/test_pipeline.py tests/test_golden.py tests/test_fast_mode.py tests/test_keyframes.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk']
print(f\"{sys.argv[2]:22s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  direct {b['direct']['avg_ms']*1e3:6.2f} us/frame  lk {b['lkalign']['avg_ms']*1e3:7.1f} us/batch  parity {d['parity_vs_oracle']['max_rel_frobenius'] if 'parity_vs_oracle' in d else '-'}\")" $1 $2; }
for rep in 1 2; do
for lib in prod base; do
  if [ $lib = base ]; then export VISO_LIB=$B; else unset VISO_LIB; fi
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-svo --rig-steps 0 > $OUT/${lib}_d$rep.json 2> $OUT/${lib}_d$rep.err || { tail -20 $OUT/${lib}_d$rep.err; exit 1; }
  summ $OUT/${lib}_d$rep.json "$lib-driverargs"
  timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 > $OUT/${lib}_f$rep.json 2> $OUT/${lib}_f$rep.err || { tail -20 $OUT/${lib}_f$rep.err; exit 1; }
  summ $OUT/${lib}_f$rep.json "$lib-default"
done
done
