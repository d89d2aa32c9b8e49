#!/bin/bash
# Experiment pass (dev): bench line without the CPU / SVO legs, the direct-pose
# tests, and the phase probe when the probe library is built.
set -o pipefail
T=${1:-exp1}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-svo --no-cpu > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_track.py tests/test_rig_direct.py tests/test_pipeline.py tests/test_golden.py tests/test_keyframes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
if [ -f viso_amd/libviso_amd_probe.so ]; then
  timeout -k 10 120 python -u tools/probe_direct.py > gpurun_out/$T/probe.log 2>&1 || { tail -20 gpurun_out/$T/probe.log; exit 1; }
  sed -n 7,20p gpurun_out/$T/probe.log
fi
python -c "
import json;d=json.loads(open('gpurun_out/$T/bench.json').read());print(d['value'],d['kernels_breakdown_chunk'],d['other_precision']['value'], d['rig_direct']['faithful']['timesteps_per_s'], d['rig_direct']['fast']['timesteps_per_s'])"
