#!/bin/bash
# Dev experiment: level-1 pyramid launch with unused dynamic LDS per block (limits blocks per CU).
# (The VISO_EXP_PYR_LDS hook this script drives was removed after the experiment; see DESIGN.md, round-3 log.)
set -o pipefail
OUT=gpurun_out/${1:-pyrlds}
mkdir -p $OUT
export TMPDIR=/tmp
for n in 20 50 128; do
for L in 0 16384 32768 49152; do
  VISO_EXP_PYR_LDS=$L IMAGES=$n REPS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k${n}_$L -o run -- python -u tools/bench_pyramid.py > $OUT/k${n}_$L.log 2>&1 || { tail -20 $OUT/k${n}_$L.log; exit 1; }
  python tools/db2stats.py $OUT/k${n}_$L/run_results.db $OUT/k${n}_$L.csv
  python - $OUT/k${n}_$L.csv $n $L <<'PY'
import csv, sys
r = {row["Name"]: row for row in csv.DictReader(open(sys.argv[1]))}
a = [v for k, v in r.items() if "pyr_down_sk" in k][0]; b = [v for k, v in r.items() if "pyr_tail" in k][0]
print(f"images {sys.argv[2]:>4} lds {sys.argv[3]:>6}: L1 {float(a['AverageNs'])/1e3:6.2f} us (min {float(a['MinNs'])/1e3:6.2f})  tail {float(b['AverageNs'])/1e3:6.2f} us")
PY
done
done
