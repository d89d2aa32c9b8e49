#!/bin/bash
# Round-3 dev step: LK/KLT parity, direct-pose ring probe, bench lines of the
# product library and of an experiment variant library ($2).
set -o pipefail
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_track.py tests/test_pipeline.py tests/test_golden.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe.log 2>&1 || { echo "probe failed"; tail -20 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2],'value',d['value'],'ms/step',d['ms_per_step'],'breakdown',d['kernels_breakdown_chunk'])" $1 $2; }
for prec in faithful fast; do
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision $prec > $OUT/b_$prec.json 2> $OUT/b_$prec.err || { tail -20 $OUT/b_$prec.err; exit 1; }
summ $OUT/b_$prec.json $prec
if [ -n "$2" ]; then
VISO_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision $prec > $OUT/bx_$prec.json 2> $OUT/bx_$prec.err || { tail -20 $OUT/bx_$prec.err; exit 1; }
summ $OUT/bx_$prec.json "variant-$prec"
fi
done
