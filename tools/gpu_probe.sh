#!/bin/bash
# Direct-pose phase probe (needs viso_amd/libviso_amd_probe.so: VISO_VARIANT=probe python viso_amd/build.py)
set -o pipefail
T=${1:-probe}
mkdir -p gpurun_out/$T
timeout -k 10 120 python -u tools/probe_direct.py > gpurun_out/$T/probe.log 2>&1 || { tail -20 gpurun_out/$T/probe.log; exit 1; }
cat gpurun_out/$T/probe.log
