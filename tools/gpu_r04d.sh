# init-path (1,024-thread normalise / compaction, gated frames skip the
# RANSAC body) and LK alignment shared bilinear weights: parity tests, the
# driver-argument bench, and the same under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_00_configs.py tests/test_pipeline.py tests/test_golden.py tests/test_geometry.py tests/test_track.py tests/test_stereo_init.py tests/test_kitti_e2e.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/bench_prof.json 2> $OUT/bench_prof.err
