#!/bin/bash
# Dev: kernel-argument placement experiment (HIP_FORCE_DEV_KERNARG=1 vs the
# default) on the rig probe and the bench's faithful line.
set -o pipefail
OUT=gpurun_out/${1:-karg}
mkdir -p $OUT
export TMPDIR=/tmp
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 120 python -u tools/probe_rig.py > $OUT/rig_$k.log 2>&1 || { tail -20 $OUT/rig_$k.log; exit 1; }
  echo "== HIP_FORCE_DEV_KERNARG=$k"; sed -n 3,8p $OUT/rig_$k.log; tail -1 $OUT/rig_$k.log
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 > $OUT/b_$k.json 2> $OUT/b_$k.err || { tail -20 $OUT/b_$k.err; exit 1; }
  python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk'];print(d['value'], b['direct']['avg_ms']*1e3, b['lkalign']['avg_ms']*1e3)" $OUT/b_$k.json
done
