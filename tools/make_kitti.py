#!/usr/bin/env python3
"""Write a KITTI-odometry-layout copy of the synthetic stereo sequence (dev tool):
<out>/sequences/NN/{image_0,image_1}/%06d.png + calib.txt, for exercising
bench.py --kitti / viso_amd.kitti on machines without the KITTI dataset.

usage: make_kitti.py OUT N_FRAMES [N_SEQUENCES]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import PIL.Image

    from viso_amd.shard import sequence_seed
    from viso_amd.synth import Sequence

    out, n = sys.argv[1], int(sys.argv[2])
    n_seq = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    for s in range(n_seq):
        seq = Sequence(1242, 375, seed=sequence_seed(s))
        root = os.path.join(out, "sequences", f"{s:02d}")
        for cam in (0, 1):
            os.makedirs(os.path.join(root, f"image_{cam}"), exist_ok=True)
            for f in range(n):
                PIL.Image.fromarray(seq.image(f, cam)).save(os.path.join(root, f"image_{cam}", f"{f:06d}.png"))
        fx, fy, cx, cy = seq.K
        P0 = [fx, 0, cx, 0, 0, fy, cy, 0, 0, 0, 1, 0]
        P1 = [fx, 0, cx, -fx * seq.p.baseline, 0, fy, cy, 0, 0, 0, 1, 0]
        with open(os.path.join(root, "calib.txt"), "w") as fh:
            for k, P in enumerate((P0, P1, P0, P1)):
                fh.write(f"P{k}: " + " ".join(f"{v:.12e}" for v in P) + "\n")
        print(root, n, "pairs")


if __name__ == "__main__":
    main()
