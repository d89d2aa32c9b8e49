#!/bin/bash
# Round-3 GPU step: init-frame geometry kernel times (rocprofv3 over the
# geometry / pipeline GPU tests) and a roctx marker trace of a short bench.
set -o pipefail
OUT=gpurun_out/${1:-geo3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/geo -o run -- python -u -m pytest tests/test_geometry.py tests/test_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/geo.log 2>&1 || { tail -20 $OUT/geo.log; exit 1; }
tail -1 $OUT/geo.log
python tools/db2stats.py $(find $OUT/geo -name '*results.db' | head -1) $OUT/geo_kernel_stats.csv
grep -E "recover|h_refine|h_moment|Name" $OUT/geo_kernel_stats.csv | cut -c1-160
VISO_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace -d $OUT/roctx -o run -- python -u bench.py --no-cpu --no-svo --rig-steps 4 --steps 20 --warmup 5 > $OUT/roctx_bench.json 2> $OUT/roctx_bench.err || { echo "roctx run failed"; tail -30 $OUT/roctx_bench.err; exit 1; }
python - $OUT <<'PY'
import glob, sqlite3, sys, collections
db = glob.glob(f"{sys.argv[1]}/roctx/**/*results.db", recursive=True)[0]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
mt = [t for t in tabs if 'region' in t.lower() or 'marker' in t.lower()]
print("tables with markers:", mt)
for t in mt:
    cols = [r[1] for r in c.execute(f"pragma table_info('{t}')")]
    if 'name' in cols and 'start' in cols and 'end' in cols:
        cnt = collections.Counter(); dur = collections.Counter()
        has_ext = 'extdata' in cols
        q = f"select {'extdata' if has_ext else 'name'}, start, end from '{t}'"
        for n, s, e in c.execute(q):
            if has_ext:
                import json
                n = json.loads(n).get("message", n)
            cnt[n] += 1; dur[n] += (e - s)
        for n in sorted(cnt, key=lambda k: -dur[k])[:12]:
            print(f"  {t}: {n:22s} n={cnt[n]:6d} mean {dur[n] / cnt[n] / 1e3:9.2f} us")
        break
PY
