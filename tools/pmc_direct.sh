#!/bin/bash
# PMC pass over the direct-pose kernels (dev tool, via gpurun): bash tools/pmc_direct.sh TAG [bench args]
set -o pipefail
TAG=${1:-pmcd}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --no-svo --rig-steps 0 --steps 100 --warmup 10 $@"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $OUT/a -o run --output-format csv -- $B > $OUT/a.log 2>&1 || { echo "pass a failed"; tail -20 $OUT/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d $OUT/b -o run --output-format csv -- $B > $OUT/b.log 2>&1 || { echo "pass b failed"; tail -20 $OUT/b.log; exit 1; }
python tools/pmc_summary.py $OUT/a $OUT/b
