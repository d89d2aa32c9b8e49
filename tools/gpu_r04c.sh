# full GPU suite on HEAD (+ row_ror tree levels), the driver-argument bench,
# the boundary ubench (GPU-side boundary with long kernels / graphs) and the
# FAST tile-height variants under rocprofv3
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread --durations=25 -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err && \
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --no-config2 --no-init > $OUT/bench_default.json 2> $OUT/bench_default.err && \
timeout -k 10 60 ./tools/ubench/boundary_bench > $OUT/boundary_bench.jsonl 2>&1 && \
for v in "" _ft4 _ft16; do
  VISO_LIB=$PWD/viso_amd/libviso_amd$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof$v -o fast -- python3 tools/bench_fast.py > $OUT/fast$v.log 2>&1 || exit 1
done
