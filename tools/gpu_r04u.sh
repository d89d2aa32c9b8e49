# background LK: the ready-flag poll interval (s_sleep 4 / 32 / 127 quanta)
set -o pipefail
export TMPDIR=/tmp
TESTS="tests/test_golden.py" bash tools/gpu_ab3.sh r04u viso_amd/libviso_amd.so viso_amd/libviso_amd_poll32.so viso_amd/libviso_amd_poll127.so
