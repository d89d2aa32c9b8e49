#!/bin/bash
# Dev A/B: a variant library ($2) under the direct-pose / pipeline GPU tests,
# then bench lines (default and the driver's arguments) for product and variant.
set -o pipefail
OUT=gpurun_out/${1:-vab}
V=$2
mkdir -p $OUT
export TMPDIR=/tmp
VISO_LIB=$V timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_pipeline.py tests/test_golden.py tests/test_fast_mode.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d.get('kernels_breakdown_chunk') or {}
print(f\"{sys.argv[2]:18s} {d['value']:9.1f} frames/s  ms/step {d['ms_per_step']:.4f}  \" + '  '.join(f'{k} {v[\"avg_ms\"]*1e3:.1f}' for k, v in b.items()) + f\"  parity {(d.get('parity_vs_oracle') or {}).get('max_rel_frobenius')}\")" $1 $2; }
for rep in 1 2; do
for lib in prod var; do
  if [ $lib = var ]; then export VISO_LIB=$V; else unset VISO_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 > $OUT/${lib}_f$rep.json 2> $OUT/${lib}_f$rep.err || { tail -20 $OUT/${lib}_f$rep.err; exit 1; }
  summ $OUT/${lib}_f$rep.json "$lib-default"
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-svo --rig-steps 0 > $OUT/${lib}_d$rep.json 2> $OUT/${lib}_d$rep.err || { tail -20 $OUT/${lib}_d$rep.err; exit 1; }
  summ $OUT/${lib}_d$rep.json "$lib-driverargs"
done
done
