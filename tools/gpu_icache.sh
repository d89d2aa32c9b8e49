#!/bin/bash
# Dev: instruction-cache counters of the direct-pose kernels (one rocprofv3 --pmc pass).
set -o pipefail
OUT=gpurun_out/${1:-icache}
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --no-cpu --no-svo --rig-steps 0 --steps 64 --warmup 10 --batch 64"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU -d $OUT/ic -o run --output-format csv -- $B > $OUT/ic.log 2>&1 || { echo "ic failed"; tail -20 $OUT/ic.log; exit 1; }
python - $OUT <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"{sys.argv[1]}/ic/run_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0].replace("void viso::(anonymous namespace)::", "")
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "direct_level" in k or "lk_align" in k or "rig_level" in k:
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()}, "dispatch-values", len(next(iter(d.values()))))
PY
