# Dev iteration on the GPU box (via gpurun from the repo root): selected GPU
# tests (default: the tracking path), the direct-pose probe, one bench line
# per precision.  Usage: bash tools/gpu_iter.sh TAG [pytest selectors...]
set -o pipefail
TAG=${1:-iter}; shift
SEL=${@:-tests/test_track.py tests/test_pipeline.py tests/test_golden.py tests/test_stereo_init.py tests/test_keyframes.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
if [ -n "$PROBE" ]; then
  timeout -k 10 120 python -u tools/probe_direct.py > $OUT/probe.log 2>&1 && head -16 $OUT/probe.log
fi
if [ -n "$BENCH" ]; then
for prec in faithful fast; do
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision $prec > $OUT/b_$prec.json 2> $OUT/b_$prec.err || { tail -20 $OUT/b_$prec.err; exit 1; }
python -c "
import json;d=json.loads(open('$OUT/b_$prec.json').read().strip().splitlines()[-1])
print('$prec value',d['value'],'ms/step',d['ms_per_step'],'breakdown',d['kernels_breakdown_chunk'])"
done
fi
