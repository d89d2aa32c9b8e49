#!/bin/bash
# Round-3 GPU step: rig / facade tests and a roctx marker trace of a short bench.
set -o pipefail
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rig_direct.py tests/test_stereo_abi.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
VISO_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $OUT/roctx -o run -- python -u bench.py --no-cpu --no-svo --rig-steps 8 --steps 20 --warmup 5 > $OUT/roctx_bench.json 2> $OUT/roctx_bench.err || { echo "roctx run failed"; tail -30 $OUT/roctx_bench.err; exit 1; }
ls -R $OUT/roctx | head
