#!/bin/bash
# Dev: direct / rig check: their GPU tests, the rig probe, A/B bench lines
# (tools/gpu_ab.sh) and the rig bench (tools/gpu_rig_merge.sh kernel stats).
set -o pipefail
T=${1:-dr}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe_rig.py > gpurun_out/$T/rig_probe.log 2>&1 || { tail -20 gpurun_out/$T/rig_probe.log; exit 1; }
sed -n 3,11p gpurun_out/$T/rig_probe.log; tail -1 gpurun_out/$T/rig_probe.log
timeout -k 10 120 python -u tools/probe_direct.py > gpurun_out/$T/direct_probe.log 2>&1 || { tail -20 gpurun_out/$T/direct_probe.log; exit 1; }
grep -E "partials reduced|solve done|after B2|last block exit|boundary|entry-to-entry" gpurun_out/$T/direct_probe.log
TESTS="tests/test_pipeline.py tests/test_fast_mode.py tests/test_golden.py" bash tools/gpu_ab.sh ${T}_ab || exit 1
bash tools/gpu_rig_merge.sh ${T}_rig
