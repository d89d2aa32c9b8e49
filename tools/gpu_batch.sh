#!/bin/bash
# Dev: the bench line at several ingest batch sizes (frames per chunk).
set -o pipefail
OUT=gpurun_out/${1:-batch}
mkdir -p $OUT
export TMPDIR=/tmp
for b in 50 100 128; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-svo --rig-steps 0 --batch $b --steps 256 > $OUT/b$b.json 2> $OUT/b$b.err || { tail -20 $OUT/b$b.err; exit 1; }
  python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b=d['kernels_breakdown_chunk'];print(sys.argv[2], d['value'], d['other_precision']['value'], 'frac', d['roofline']['frac'], 'pyr', b['pyramid']['avg_ms']*1e3, 'lk', b['lkalign']['avg_ms']*1e3, 'direct', b['direct']['avg_ms']*1e3)" $OUT/b$b.json $b
done
