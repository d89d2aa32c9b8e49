#!/bin/bash
# Experiment pass against an alternative library build (dev):
#   VISO_VARIANT=<v> python viso_amd/build.py, then bash tools/gpu_exp_lib.sh <tag> viso_amd/libviso_amd_<v>.so
set -o pipefail
T=${1:-expl}
export VISO_LIB=$2
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u bench.py --no-svo --no-cpu > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_track.py tests/test_rig_direct.py tests/test_pipeline.py tests/test_stereo_init.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
python -c "
import json;d=json.loads(open('gpurun_out/$T/bench.json').read());print(d['value'],d['kernels_breakdown_chunk'],d['other_precision']['value'], d['rig_direct']['faithful']['timesteps_per_s'], d['rig_direct']['fast']['timesteps_per_s'])"
