#!/bin/bash
# Round-3 GPU step: facade test + direct-pose phase probe (faithful, fast).
set -o pipefail
OUT=gpurun_out/${1:-r03c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stereo_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe.log 2>&1 || { echo "probe failed"; tail -20 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
PRECISION=fast timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe_fast.log 2>&1 || { echo "probe fast failed"; tail -20 $OUT/probe_fast.log; exit 1; }
cat $OUT/probe_fast.log
