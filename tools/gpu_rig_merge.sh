#!/bin/bash
# Rig final-solve merge check: rig/facade GPU tests, two rig bench runs, kernel stats.
set -o pipefail
OUT=gpurun_out/${1:-rigm}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rig_direct.py tests/test_stereo_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-svo > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { echo "bench failed"; tail -30 $OUT/bench_$rep.err; exit 1; }
python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d['value'], {k:v for k,v in d.items() if 'rig' in k})" $OUT/bench_$rep.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u bench.py --no-cpu --no-svo > $OUT/bench_rocprof.json 2> $OUT/bench_rocprof.err || { echo "rocprof failed"; tail -30 $OUT/bench_rocprof.err; exit 1; }
python tools/db2stats.py $(find $OUT/prof -name '*results.db' | head -1) $OUT/bench_kernel_stats.csv && grep -i -E "rig|direct_level" $OUT/bench_kernel_stats.csv
