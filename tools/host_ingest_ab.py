"""host_ingest leg (bench.py measure_host_ingest: viso_process_frame per frame
from host memory) A/B inside one process: each variant is a set of
environment variables the library reads at context creation (e.g.
VISO_HOST_LK=batch), run REPS times, alternating; the poses of every run
are compared with the oracle's (computed once).  Also times a plain 466 KB
host copy into pinned memory (the copy's floor on this host).
Usage (GPU box): python tools/host_ingest_ab.py REPS 'A:' 'B:VISO_HOST_LK=batch' ..."""
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from tests import oracle_lib
    from viso_amd.synth import Sequence
    reps = int(sys.argv[1])
    variants = []
    for v in sys.argv[2:]:
        name, _, env = v.partition(":")
        variants.append((name, dict(kv.split("=", 1) for kv in env.split(",") if kv)))
    W, H = 1242, 375
    seq = Sequence(W, H, seed=0)
    per = int(os.environ.get("FRAMES", "32"))
    n = 1 + 4 + 2 * per
    left = np.stack([seq.image(f, 0) for f in range(n)])
    right = np.stack([seq.image(f, 1) for f in range(n)])
    # the copy floor: numpy -> pinned
    pin = torch.empty(W * H, dtype=torch.uint8).pin_memory().numpy()
    src = left[7].reshape(-1)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        np.copyto(pin, src)
        ts.append(time.perf_counter() - t0)
    print(f"pinned copy of {W * H} B: median {1e6 * np.median(ts):.1f} us", flush=True)
    ov = oracle_lib.Viso(seq.K, W, H, enable_tracking=1)
    ov.set_stereo(seq.p.baseline, 128, 1)
    for f in range(n):
        ov.on_new_stereo(left[f], right[f])
    oP = ov.poses()
    args = SimpleNamespace()
    for r in range(reps):
        for name, env in variants:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                out = bench.measure_host_ingest(args, seq, W, H, left, right, lambda *a: None, n=per)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            hP = out["_poses"]
            m = min(len(hP), len(oP))
            rel = float((np.linalg.norm(hP[:m] - oP[:m], axis=1) / np.linalg.norm(oP[:m], axis=1)).max())
            sp = {k: v["us_per_frame"] for k, v in out["split_us_per_frame"].items()}
            print(f"rep {r} {name:10s}: {out['us_per_frame']:6.1f} us/frame, host enqueue "
                  f"{out['host_enqueue_us_per_frame']:5.1f}, sync {out['sync_us']:7.1f}, split {sp}, "
                  f"parity {m} frames rel {rel:.1e}", flush=True)


if __name__ == "__main__":
    main()
