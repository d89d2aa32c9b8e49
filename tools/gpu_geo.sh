set -o pipefail
mkdir -p gpurun_out/geo
timeout -k 10 300 python -u -m pytest tests/test_geometry.py tests/test_golden.py tests/test_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/geo/pytest.log 2>&1 || { tail -30 gpurun_out/geo/pytest.log; exit 1; }
tail -2 gpurun_out/geo/pytest.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/geo/prof -o run -- python -u -m pytest tests/test_geometry.py -m gpu -x -q > gpurun_out/geo/prof.log 2>&1 || { tail -20 gpurun_out/geo/prof.log; exit 1; }
f=$(find gpurun_out/geo/prof -name '*kernel_stats.csv' | head -1); grep -E "recover|h_refine|h_moment|Name" $f | cut -c1-160
