"""configs[2] tracking leg alone (bench.py measure_config2 part 1), repeated:
the monocular reference initialisation at 1920x1080, then 16 tracking frames
in one batched call, host clock around the call.  Usage (GPU box):
python tools/c2_track.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from viso_amd.synth import Sequence
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    W, H, n_track = 1920, 1080, 16
    seq = Sequence(W, H, seed=0, block_m=0.35)
    left = np.stack([seq.image(f, 0) for f in range(6 + n_track)])
    d_left = torch.from_numpy(left).cuda()
    torch.cuda.synchronize()
    for r in range(reps):
        v, per, n_init, dt = bench.run_reference_init(seq, W, H, d_left, 6, n_track, n_track, timing=False)
        print(f"rep {r}: init {np.mean(per[1:]):.1f} us/frame, tracking {n_track / dt:.1f} frames/s "
              f"({1e6 * dt / n_track:.1f} us/frame), state {v.state}", flush=True)
        v.close()


if __name__ == "__main__":
    main()
