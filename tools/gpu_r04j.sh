# round-4 evidence on HEAD: the default bench line, and the driver-argument
# bench under rocprofv3 --kernel-trace --stats (kernel durations for profiles/)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
echo default ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err; exit 1; }
echo prof ok
find $OUT/prof -name "*.csv" -o -name "*.db" | head
