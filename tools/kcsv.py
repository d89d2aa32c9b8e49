"""Summarise a rocprofv3 --stats kernel_stats.csv: name (shortened), calls, avg us, total ms."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"]
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", name)
    short = (m.group(1) + (m.group(2) or "")) if m else name[:40]
    print(f"{short:40s} {int(r['Calls']):6d} avg {float(r['AverageNs']) / 1e3:9.2f} us  "
          f"tot {int(r['TotalDurationNs']) / 1e6:8.3f} ms")
