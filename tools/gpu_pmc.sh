#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own kill timeout):
#  gn_occ  : occupancy / instruction mix of the direct-pose GN kernels (bench.py tracking path)
#  svo_f/w : HBM FETCH_SIZE / WRITE_SIZE of the stereo-VO feature and matching kernels (tools/bench_svo.py)
#  svo_sq  : their instruction mix / VALU busy (the matching pass is VALU/latency-bound, not HBM-bound)
# Usage (via gpurun, from the repo root): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --no-svo --rig-steps 0 --steps 100 --warmup 20"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/gn_occ -o run --output-format csv -- $B > $OUT/gn_occ.log 2>&1 || { echo "gn_occ failed"; tail -20 $OUT/gn_occ.log; exit 1; }
echo gn_occ ok
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/svo_f -o run --output-format csv -- python -u tools/bench_svo.py > $OUT/svo_f.log 2>&1 || { echo "svo_f failed"; tail -20 $OUT/svo_f.log; exit 1; }
echo svo_f ok
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/svo_w -o run --output-format csv -- python -u tools/bench_svo.py > $OUT/svo_w.log 2>&1 || { echo "svo_w failed"; tail -20 $OUT/svo_w.log; exit 1; }
echo svo_w ok
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/svo_sq -o run --output-format csv -- python -u tools/bench_svo.py > $OUT/svo_sq.log 2>&1 || { echo "svo_sq failed"; tail -20 $OUT/svo_sq.log; exit 1; }
echo svo_sq ok
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d $OUT/gn_f64 -o run --output-format csv -- $B > $OUT/gn_f64.log 2>&1 || { echo "gn_f64 failed (counters may not exist)"; tail -20 $OUT/gn_f64.log; exit 0; }
echo gn_f64 ok
find $OUT -name '*.csv' | head
