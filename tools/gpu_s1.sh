#!/bin/bash
# Dev: the GPU suite, then an A/B of the product library against others
# (tools/gpu_ab3.sh).  usage: gpu_s1.sh OUT lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TESTS=tests/test_golden.py bash tools/gpu_ab3.sh $(basename $O)_ab "$@"
