set -o pipefail
mkdir -p gpurun_out/svo1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_svo.py tests/test_kitti_e2e.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/svo1/pytest.log 2>&1 || { tail -30 gpurun_out/svo1/pytest.log; exit 1; }
tail -2 gpurun_out/svo1/pytest.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/svo1/svo_f -o run --output-format csv -- python -u tools/bench_svo.py > gpurun_out/svo1/svo_f.log 2>&1 || { tail -20 gpurun_out/svo1/svo_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/svo1/svo_w -o run --output-format csv -- python -u tools/bench_svo.py > gpurun_out/svo1/svo_w.log 2>&1 || { tail -20 gpurun_out/svo1/svo_w.log; exit 1; }
timeout -k 10 200 python -u tools/bench_svo.py 2>&1 | tail -3
