# config tests incl. the three LK forms (background / leftovers+drain / batched)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04r
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_00_configs.py -x -v --timeout 120 --timeout-method thread --durations=0 -m gpu > $OUT/configs.log 2>&1 || { tail -40 $OUT/configs.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/configs.log | tail -12
