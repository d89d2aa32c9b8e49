#!/bin/bash
# Quick GPU iteration (dev tool, via gpurun from the repo root):
#   bash tools/gpu_quick.sh TAG [pytest selectors...]
# GPU parity tests (default: all -m gpu), the direct-pose phase probe
# (needs viso_amd/libviso_amd_probe.so), and one bench line without the CPU legs.
set -o pipefail
TAG=${1:-quick}; shift
SEL=${@:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $SEL -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
if [ -f viso_amd/libviso_amd_probe.so ]; then
  timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe.log 2>&1 || { echo "probe failed"; tail -20 $OUT/probe.log; exit 1; }
  cat $OUT/probe.log
fi
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value',d['value'],'ms/step',d['ms_per_step'],'kernels',d['kernels'],'breakdown',d['kernels_breakdown_chunk'])"
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision fast > $OUT/bench_fast.json 2> $OUT/bench_fast.err || { echo "bench fast failed"; tail -20 $OUT/bench_fast.err; exit 1; }
python -c "
import json;d=json.loads(open('$OUT/bench_fast.json').read().strip().splitlines()[-1])
print('FAST value',d['value'],'ms/step',d['ms_per_step'],'kernels',d['kernels'],'breakdown',d['kernels_breakdown_chunk'])"
