"""The host-frame path alone (bench.py measure_host_ingest's calls, dev tool):
frame 0's stereo pair initialises, then N frames through viso_process_frame
from host memory, one synchronize.  For rocprofv3 timelines (host_timeline.py).
usage: python tools/host_ingest_run.py [N=48]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import viso_amd
    from viso_amd.synth import Sequence
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    W, H = 1242, 375
    seq = Sequence(W, H, seed=0)
    left = [seq.image(f, 0) for f in range(n + 1)]
    right0 = seq.image(0, 1)
    v = viso_amd.Viso(*seq.K, width=W, height=H, enable_tracking=1)
    v.set_stereo(seq.p.baseline, 128, 1)
    v.process(left[0], right0)
    v.synchronize()
    t0 = time.perf_counter()
    for f in range(1, n + 1):
        v.OnNewFrame(left[f])
    t1 = time.perf_counter()
    v.synchronize()
    t2 = time.perf_counter()
    print(f"{n} frames: enqueue {1e6 * (t1 - t0) / n:.1f} us/frame, total {1e6 * (t2 - t0) / n:.1f} us/frame")
    v.close()


if __name__ == "__main__":
    main()
