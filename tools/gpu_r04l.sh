# background LK alignment with the end-of-chunk drain (12-wave direct pose +
# lk_item_kernel resident beside it): parity tests under that library, then
# the A/B against the product library (16-wave direct, LK batch after the chain)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
VISO_LIB=$PWD/viso_amd/libviso_amd_bg.so timeout -k 10 300 python -u -m pytest tests/test_00_configs.py tests/test_pipeline.py tests/test_golden.py tests/test_fast_mode.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_bg.log 2>&1 || { tail -40 $OUT/pytest_bg.log; exit 1; }
tail -1 $OUT/pytest_bg.log
TESTS="tests/test_track.py" bash tools/gpu_ab3.sh r04l viso_amd/libviso_amd.so viso_amd/libviso_amd_bg.so viso_amd/libviso_amd_bgp.so
