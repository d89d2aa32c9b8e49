#!/bin/bash
# Dev experiment: LK alignment beside the direct chain (side stream, CU split).
# (The VISO_EXP_* hooks this script drives were removed after the experiment; see DESIGN.md, round-3 log.)
set -o pipefail
OUT=gpurun_out/${1:-lkov}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; return 1; }
  python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk'];print(sys.argv[2], d['value'], d['other_precision']['value'], 'direct', round(b['direct']['avg_ms']*1e3,2), 'lk', round(b['lkalign']['avg_ms']*1e3,1), b['lkalign']['launches'])" $OUT/$tag.json $tag
}
run base VISO_NOOP=1 || exit 1
run side VISO_EXP_LK_SIDE=1 || exit 1
run cu64_g192 VISO_EXP_LK_CUS=64 VISO_EXP_DIRECT_GROUPS=192 || exit 1
run cu48_g208 VISO_EXP_LK_CUS=48 VISO_EXP_DIRECT_GROUPS=208 || exit 1
run cu80_g176 VISO_EXP_LK_CUS=80 VISO_EXP_DIRECT_GROUPS=176 || exit 1
run g192_only VISO_EXP_DIRECT_GROUPS=192 || exit 1
