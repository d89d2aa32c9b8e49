"""Print the headline numbers of bench.py JSON lines (dev tool):
  python tools/bline.py out1.json [out2.json ...]"""
import json
import sys

for p in sys.argv[1:]:
    try:
        d = json.loads(open(p).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(p, "unreadable:", e)
        continue
    kb = d.get("kernels_breakdown_chunk") or {}
    hi = d.get("host_ingest") or {}
    ip = d.get("init_path") or {}
    par = d.get("parity_vs_oracle") or {}
    print(p, f"value {d.get('value')} ms/step {d.get('ms_per_step')}",
          f"direct {json.dumps(kb.get('direct'))[:90]}",
          f"roof {d.get('roofline', {}).get('frac')}",
          f"host_ingest {hi.get('us_per_frame')} init {ip.get('init_frame_us')} detect {ip.get('detect_frame_us')}",
          f"parity {par.get('max_rel_frobenius')} ({par.get('frames')} frames)")
