# background LK: the config-1 test with the side stream on its own queue
# (CU-masked) and on a plain (shared) stream, background off for reference
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
T="tests/test_00_configs.py::test_gpu_config1_bench_workload_matches_oracle"
VISO_LK_BG=0 timeout -k 10 200 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/nobg.log 2>&1; echo "nobg rc=$?"; tail -1 $OUT/nobg.log
VISO_LK_QUEUE=shared timeout -k 10 200 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/shared.log 2>&1; echo "shared rc=$?"; tail -1 $OUT/shared.log; grep -m3 "^E " $OUT/shared.log
timeout -k 10 200 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/masked.log 2>&1; echo "masked rc=$?"; tail -1 $OUT/masked.log; grep -m3 "^E " $OUT/masked.log
true
