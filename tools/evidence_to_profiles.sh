#!/bin/bash
# Copy one evidence pass (tools/gpu_evidence.sh TAG, merged back into
# gpurun_out/) into the round's committed profiles/.  usage: evidence_to_profiles.sh TAG ROUND
set -e
TAG=$1; R=${2:-r06}; IN=gpurun_out/$TAG
cp $IN/pytest_gpu.log profiles/${R}_pytest_gpu.log
cp $IN/smoke.log profiles/${R}_smoke.log
tail -1 $IN/bench_driver.json > profiles/${R}_bench_line_driver_args.json
tail -1 $IN/bench_default.json > profiles/${R}_bench_line_default.json
cp $IN/kernel_stats_nobg.csv profiles/${R}_direct_kernel_stats.csv
cp $IN/kernel_stats.csv profiles/${R}_bench_kernel_stats.csv
SRC_HASH=$(cat $IN/src.txt) python tools/pmc_kernels.py gpurun_out/${TAG}_pmc profiles/${R}_gn_svo_pmc.json
cp $IN/src.txt profiles/${R}_evidence_src.txt
cp gpurun_out/${TAG}_pyr/pyramid_traffic.json profiles/pyramid_traffic.json
for f in direct_probe_bg direct_probe_nobg lk_items_probe; do
  [ -f $IN/$f.log ] && cp $IN/$f.log profiles/${R}_$f.log
done
echo "profiles/${R}_* updated from $IN"
