# PMC refresh on HEAD: tools/gpu_pmc.sh's passes, plus the
# driver-argument bench (one 20-frame chunk) under the occupancy counters and
# the wait-state counters, for lk_align_kernel / direct_level_kernel there
set -o pipefail
export TMPDIR=/tmp
# counter collection serialises dispatches: the chunk-resident background LK
# grid would wait out its flag timeouts, so the passes run the batched LK path
export VISO_LK_BG=0
bash tools/gpu_pmc.sh r04pmc || exit 1
OUT=gpurun_out/r04pmc
B20="python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-svo --rig-steps 0 --no-init --no-config2 --no-other"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/d20_occ -o run --output-format csv -- $B20 > $OUT/d20_occ.log 2>&1 || { echo "d20_occ failed"; tail -20 $OUT/d20_occ.log; exit 1; }
echo d20_occ ok
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM -d $OUT/d20_wait -o run --output-format csv -- $B20 > $OUT/d20_wait.log 2>&1 || { echo "d20_wait failed"; tail -20 $OUT/d20_wait.log; exit 1; }
echo d20_wait ok
