set -o pipefail
mkdir -p gpurun_out/exp1
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-svo --no-cpu > gpurun_out/exp1/bench.json 2> gpurun_out/exp1/bench.err || { tail -20 gpurun_out/exp1/bench.err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_track.py tests/test_rig_direct.py tests/test_pipeline.py tests/test_golden.py tests/test_keyframes.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/exp1/pytest.log 2>&1; tail -15 gpurun_out/exp1/pytest.log
