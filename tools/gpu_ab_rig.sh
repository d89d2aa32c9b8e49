#!/bin/bash
# Dev A/B: bench faithful/fast lines and the rig for the product and a variant library ($2).
set -o pipefail
OUT=gpurun_out/${1:-abr}
V=$2
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk'];r=d['rig_direct']
print(f\"{sys.argv[2]:8s} {d['value']:9.1f} / {d['other_precision']['value']:9.1f} frames/s  direct {b['direct']['avg_ms']*1e3:6.2f} us/frame  rig {r['faithful']['timesteps_per_s']} / {r['fast']['timesteps_per_s']}\")" $1 $2; }
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-svo > $OUT/p_$rep.json 2> $OUT/p_$rep.err || { tail -20 $OUT/p_$rep.err; exit 1; }
  summ $OUT/p_$rep.json prod
  VISO_LIB=$V timeout -k 10 300 python -u bench.py --no-cpu --no-svo > $OUT/v_$rep.json 2> $OUT/v_$rep.err || { tail -20 $OUT/v_$rep.err; exit 1; }
  summ $OUT/v_$rep.json var
done
