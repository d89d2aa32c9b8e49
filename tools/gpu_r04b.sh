# FAST rewrite + wave-parallel RANSAC hypotheses / scan: parity tests, then
# the driver-argument bench under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_image.py tests/test_geometry.py tests/test_00_configs.py tests/test_pipeline.py tests/test_golden.py -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 60 ./tools/ubench/boundary_bench > $OUT/boundary_bench.jsonl 2>&1
