#!/bin/bash
# One evidence pass on the GPU box for the current HEAD (round 5 on):
#   the GPU suite, smoke, the default and driver-argument bench lines, a
#   rocprofv3 kernel trace of the bench with the background LK grid OFF
#   (VISO_LK_BG=0: clean direct_level_kernel durations; with the grid on, the
#   trace's serialised bookkeeping distorts the chain) and one with it on,
#   then the PMC passes (tools/gpu_pmc.sh, grid off; tools/gpu_pyr_pmc.sh, the
#   image pass's HBM traffic over bench.py), and, when the probe
#   build is present (VISO_VARIANT=probe VISO_DEFS=-DVISO_PROBE_LIGHT), the
#   direct chain's per-level phases with the grid on and off
#   (tools/probe_direct.py) and the LK tail (tools/probe_lk_items.py).
# Usage (via gpurun, from the repo root): bash tools/gpu_evidence.sh TAG
# (tools/evidence_to_profiles.sh TAG then copies the summaries to profiles/)
set -o pipefail
TAG=${1:-evidence}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 python -c "import viso_amd._lib as l; print(l.built_hash())" > $OUT/src.txt || { echo "library hash failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench (driver args) failed"; tail -30 $OUT/bench_driver.err; exit 1; }
echo "driver-args line ok"
timeout -k 10 500 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail -30 $OUT/bench_default.err; exit 1; }
echo "default line ok"
SMALL="--no-cpu --no-svo --rig-steps 0 --no-init --no-config2 --no-other --no-host-ingest"
VISO_LK_BG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_nobg -o run -- python -u bench.py --gpus 1 --steps 20 --warmup 5 $SMALL > $OUT/bench_rocprof_nobg.json 2> $OUT/bench_rocprof_nobg.err || { echo "rocprof (grid off) failed"; tail -30 $OUT/bench_rocprof_nobg.err; exit 1; }
python tools/db2stats.py $(find $OUT/prof_nobg -name '*results.db' | head -1) $OUT/kernel_stats_nobg.csv && echo "kernel stats (grid off): $OUT/kernel_stats_nobg.csv"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u bench.py --no-cpu --svo-cpu-pairs 0 --no-host-ingest > $OUT/bench_rocprof.json 2> $OUT/bench_rocprof.err || { echo "rocprof failed"; tail -30 $OUT/bench_rocprof.err; exit 1; }
python tools/db2stats.py $(find $OUT/prof -name '*results.db' | head -1) $OUT/kernel_stats.csv && echo "kernel stats: $OUT/kernel_stats.csv"
VISO_LK_BG=0 bash tools/gpu_pmc.sh ${TAG}_pmc | tail -3
bash tools/gpu_pyr_pmc.sh ${TAG}_pyr | tail -3
if [ -f viso_amd/libviso_amd_probe.so ]; then
  VISO_LIB=$PWD/viso_amd/libviso_amd_probe.so timeout -k 10 200 python -u tools/probe_direct.py > $OUT/direct_probe_bg.log 2>&1 || { echo "direct probe failed"; tail -20 $OUT/direct_probe_bg.log; exit 1; }
  VISO_LK_BG=0 VISO_LIB=$PWD/viso_amd/libviso_amd_probe.so timeout -k 10 200 python -u tools/probe_direct.py > $OUT/direct_probe_nobg.log 2>&1 || { echo "direct probe (grid off) failed"; tail -20 $OUT/direct_probe_nobg.log; exit 1; }
  VISO_LIB=$PWD/viso_amd/libviso_amd_probe.so timeout -k 10 200 python -u tools/probe_lk_items.py > $OUT/lk_items_probe.log 2>&1 || { echo "LK probe failed"; tail -20 $OUT/lk_items_probe.log; exit 1; }
  echo "probes ok"
fi
