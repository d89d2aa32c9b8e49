#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, bench line, rocprofv3 kernel stats of the bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench (driver args) failed"; tail -30 $OUT/bench_driver.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u bench.py --no-cpu --svo-cpu-pairs 0 > $OUT/bench_rocprof.json 2> $OUT/bench_rocprof.err || { echo "rocprof failed"; tail -30 $OUT/bench_rocprof.err; exit 1; }

python tools/db2stats.py $(find $OUT/prof -name '*results.db' | head -1) $OUT/bench_kernel_stats.csv && echo "kernel stats: $OUT/bench_kernel_stats.csv"
