# SVO GPU pass: parity tests, HBM passes (FETCH_SIZE / WRITE_SIZE), kernel
# times and the bench_svo line.  Usage: bash tools/gpu_svo_check.sh TAG
set -o pipefail
T=${1:-svo1}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_svo.py tests/test_kitti_e2e.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/svo_f -o run --output-format csv -- python -u tools/bench_svo.py > $O/svo_f.log 2>&1 || { tail -20 $O/svo_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/svo_w -o run --output-format csv -- python -u tools/bench_svo.py > $O/svo_w.log 2>&1 || { tail -20 $O/svo_w.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u tools/bench_svo.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
timeout -k 10 200 python -u tools/bench_svo.py 2>&1 | tail -3
