# (1) row-layout LU of the direct solve: parity tests of the product library,
# A/B against the replicated LU; (2) background LK alignment (12-wave direct
# pose + lk_bg_kernel resident beside it): parity tests under that library,
# A/B against the product library
set -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_00_configs.py tests/test_pipeline.py tests/test_golden.py tests/test_track.py tests/test_literal_drift.py" \
  bash tools/gpu_ab3.sh r04i viso_amd/libviso_amd.so viso_amd/libviso_amd_norows.so || exit 1
OUT=gpurun_out/r04k
mkdir -p $OUT
VISO_LIB=$PWD/viso_amd/libviso_amd_bg.so timeout -k 10 300 python -u -m pytest tests/test_00_configs.py tests/test_pipeline.py tests/test_golden.py tests/test_fast_mode.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_bg.log 2>&1 || { tail -40 $OUT/pytest_bg.log; exit 1; }
tail -1 $OUT/pytest_bg.log
TESTS="tests/test_track.py" bash tools/gpu_ab3.sh r04k viso_amd/libviso_amd.so viso_amd/libviso_amd_bg.so viso_amd/libviso_amd_bgp.so
