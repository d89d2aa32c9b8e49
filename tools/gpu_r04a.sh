set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_00_configs.py -x -v --timeout 120 --timeout-method thread --durations=0 -m gpu > gpurun_out/r04a/configs.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread --durations=40 -m gpu > gpurun_out/r04a/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a/bench_driver.json 2> gpurun_out/r04a/bench_driver.err
