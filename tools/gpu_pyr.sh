export TMPDIR=/tmp
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u -m pytest tests/test_image.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
timeout -k 10 120 python -u tools/probe_pyr_tail.py > gpurun_out/$T/probe.log 2>&1 || { tail -20 gpurun_out/$T/probe.log; exit 1; }
head -12 gpurun_out/$T/probe.log
IMAGES=50 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python -u tools/bench_pyramid.py > gpurun_out/$T/rp.log 2>&1 || { tail -20 gpurun_out/$T/rp.log; exit 1; }
grep images gpurun_out/$T/rp.log
IMAGES=50 REPS=5 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d gpurun_out/$T/sq -o run -- python -u tools/bench_pyramid.py > gpurun_out/$T/sq.log 2>&1 || { tail -5 gpurun_out/$T/sq.log; exit 1; }
IMAGES=50 REPS=5 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$T/fetch -o run -- python -u tools/bench_pyramid.py > gpurun_out/$T/fetch.log 2>&1 || { tail -5 gpurun_out/$T/fetch.log; exit 1; }
IMAGES=50 REPS=5 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$T/write -o run -- python -u tools/bench_pyramid.py > gpurun_out/$T/write.log 2>&1 || { tail -5 gpurun_out/$T/write.log; exit 1; }
