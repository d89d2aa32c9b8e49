#!/bin/bash
# round-4 final evidence on HEAD (after the take-2 dequeue and leftover restructure): smoke(), the whole GPU suite, the driver-
# argument and default bench lines, and the driver-argument bench under
# rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04w}
mkdir -p $OUT
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread --durations=25 -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
echo driver ok
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
echo default ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err; exit 1; }
echo prof ok
