#!/usr/bin/env python3
"""Basic-block instruction mix of one kernel in a device assembly file (dev
tool): `hipcc --cuda-device-only -S` output, the kernel picked by a
substring of its mangled name.  Prints, per block, the instruction count,
VALU count, LDS / global memory ops and cross-lane ops, optionally only the
blocks between the first and last block containing a marker instruction.

usage: asm_blocks.py <file.s> <kernel-substring> [marker-op] [--around N]
"""
import sys


def kernel_body(lines, sub):
    st = next(i for i, l in enumerate(lines)
              if sub in l and l.split(";")[0].rstrip().endswith(":") and not l.startswith("\t"))
    en = next(i for i in range(st, len(lines)) if ".size" in lines[i] and sub in lines[i])
    return lines[st:en]


def blocks_of(body):
    out, cur, name = [], [], "entry"
    for l in body:
        t = l.strip()
        if (t.startswith(".LBB") and t.split(";")[0].rstrip().endswith(":")) or t.startswith("; %bb."):
            out.append((name, cur))
            name = t.split(":")[0] if t.startswith(".LBB") else t.split()[1].rstrip(":")
            cur = []
        elif t and not t.startswith(";") and not t.startswith("."):
            cur.append(t.split()[0])
    out.append((name, cur))
    return out


def main():
    lines = open(sys.argv[1]).read().split("\n")
    blocks = blocks_of(kernel_body(lines, sys.argv[2]))
    marker = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else None
    around = int(sys.argv[sys.argv.index("--around") + 1]) if "--around" in sys.argv else 30
    idx = range(len(blocks))
    if marker:
        hits = [i for i, (_, ops) in enumerate(blocks) if any(marker in o for o in ops)]
        if hits:
            idx = range(max(0, hits[0] - around), min(len(blocks), hits[-1] + 3))
    tot = {}
    for i in idx:
        name, ops = blocks[i]
        v = sum(o.startswith("v_") for o in ops)
        xl = sum(("permlane" in o or "_dpp" in o or "readlane" in o or "readfirstlane" in o or "bpermute" in o)
                 for o in ops)
        print(f"{i:5d} {name:12s} ops {len(ops):4d} valu {v:4d} xlane {xl:3d} ds {sum(o.startswith('ds_') for o in ops):3d} "
              f"global {sum(o.startswith('global_') or o.startswith('buffer_') for o in ops):3d} "
              f"salu {sum(o.startswith('s_') for o in ops):4d}")
        for o in ops:
            tot[o] = tot.get(o, 0) + 1
    print("mix:", ", ".join(f"{k} {n}" for k, n in sorted(tot.items(), key=lambda kv: -kv[1])[:40]))


if __name__ == "__main__":
    main()
