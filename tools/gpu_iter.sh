# Dev iteration on the GPU box (via gpurun from the repo root): the tracking-path
# parity tests, the direct-pose phase probe and one bench line per precision.
set -o pipefail
mkdir -p gpurun_out/q2
timeout -k 10 300 python -u -m pytest tests/test_track.py tests/test_pipeline.py tests/test_golden.py tests/test_stereo_init.py tests/test_keyframes.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/q2/pytest.log 2>&1 || { tail -30 gpurun_out/q2/pytest.log; exit 1; }
tail -2 gpurun_out/q2/pytest.log
timeout -k 10 120 python -u tools/probe_direct.py > gpurun_out/q2/probe.log 2>&1 && cat gpurun_out/q2/probe.log | head -12
for prec in faithful fast; do
timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --precision $prec > gpurun_out/q2/b_$prec.json 2> gpurun_out/q2/b_$prec.err || { tail -20 gpurun_out/q2/b_$prec.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/q2/b_$prec.json').read().strip().splitlines()[-1])
print('$prec value',d['value'],'ms/step',d['ms_per_step'],'breakdown',d['kernels_breakdown_chunk'], d.get('parity_vs_oracle'))"
done
