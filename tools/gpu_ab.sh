#!/bin/bash
# Dev A/B on the GPU box: bench lines (faithful, fast; no CPU / SVO / rig legs)
# and per-kernel instructions per wave for the product library and a variant
# library ($2), plus the GPU tests named in $TESTS for the product.
set -o pipefail
OUT=gpurun_out/${1:-ab}
V=$2
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
fi
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk']
print(f\"{sys.argv[2]:16s} {d['value']:9.1f} frames/s  direct {b['direct']['avg_ms']*1e3:6.2f} us/frame  lk {b['lkalign']['avg_ms']*1e3:7.1f} us/batch  pyr {b['pyramid']['avg_ms']*1e3:6.2f} us\")" $1 $2; }
for rep in 1 2; do
for prec in faithful fast; do
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision $prec > $OUT/p_${prec}_$rep.json 2> $OUT/p_${prec}_$rep.err || { tail -20 $OUT/p_${prec}_$rep.err; exit 1; }
summ $OUT/p_${prec}_$rep.json "prod-$prec"
if [ -n "$V" ]; then
VISO_LIB=$V timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision $prec > $OUT/v_${prec}_$rep.json 2> $OUT/v_${prec}_$rep.err || { tail -20 $OUT/v_${prec}_$rep.err; exit 1; }
summ $OUT/v_${prec}_$rep.json "var-$prec"
fi
done
done
if [ -n "$PMC" ]; then bash tools/gpu_pmc_insts.sh $(basename $OUT)_pmc $V | grep -A2 "gpurun_out" ; fi
