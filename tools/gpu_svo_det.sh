#!/bin/bash
# Dev: SVO detect change check: SVO GPU tests, stereo-VO bench rate, detect FETCH/WRITE per batch.
set -o pipefail
OUT=gpurun_out/${1:-svodet}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_svo.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k -o run -- python -u tools/bench_svo.py > $OUT/k.log 2>&1 || { tail -20 $OUT/k.log; exit 1; }
python tools/db2stats.py $OUT/k/run_results.db $OUT/k.csv && grep svo_ $OUT/k.csv | cut -c1-150
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/svo_f -o run --output-format csv -- python -u tools/bench_svo.py > $OUT/svo_f.log 2>&1 || { tail -5 $OUT/svo_f.log; exit 1; }
python - $OUT <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(f"{sys.argv[1]}/svo_f/run_counter_collection.csv")):
    if "svo_detect" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
        v[int(r["Dispatch_Id"])].append(float(r["Counter_Value"]))
vals = [sum(x) for x in v.values()]
print("detect FETCH_SIZE raw per dispatch (MB):", [round(x / 1024, 1) for x in vals])
PY
if [ -n "$2" ]; then
  VISO_LIB=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kv -o run -- python -u tools/bench_svo.py > $OUT/kv.log 2>&1 || { tail -20 $OUT/kv.log; exit 1; }
  python tools/db2stats.py $OUT/kv/run_results.db $OUT/kv.csv && echo "variant:" && grep svo_ $OUT/kv.csv | cut -c1-150
  VISO_LIB=$2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/svo_fv -o run --output-format csv -- python -u tools/bench_svo.py > $OUT/svo_fv.log 2>&1 || { tail -5 $OUT/svo_fv.log; exit 1; }
  python - $OUT <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(f"{sys.argv[1]}/svo_fv/run_counter_collection.csv")):
    if "svo_detect" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
        v[int(r["Dispatch_Id"])].append(float(r["Counter_Value"]))
vals = [sum(x) for x in v.values()]
print("variant detect FETCH_SIZE raw per dispatch (MB):", [round(x / 1024, 1) for x in vals])
PY
fi
