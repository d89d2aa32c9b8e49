"""Per-kernel resource usage of one csrc file from the compiler (dev tool):
VGPRs, spills, scratch, LDS, occupancy.  Usage: python tools/kres.py direct.hip [ref]
(ref = a git revision to compare against)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "viso_amd", "csrc")


def usage(path):
    cmd = ["hipcc", "-std=c++17", "-O3", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950",
           "-I", os.path.join(ROOT, "include"), "-I", CSRC, "--cuda-device-only", "-c", path,
           "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (?:\s*)([A-Za-z \[\]/]+?): (.+?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    return rows


def show(rows):
    for r in rows:
        n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        n = re.sub(r"viso::\(anonymous namespace\)::", "", n)
        print(f"{n[:70]:70s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} "
              f"vspill {r.get('VGPRs Spill','?'):>3} scratch {r.get('ScratchSize [bytes/lane]','?'):>4} "
              f"lds {r.get('LDS Size [bytes/block]','?'):>6} occ {r.get('Occupancy [waves/SIMD]','?')}")


if __name__ == "__main__":
    f = sys.argv[1]
    show(usage(os.path.join(CSRC, f)))
    if len(sys.argv) > 2:
        src = subprocess.run(["git", "show", f"{sys.argv[2]}:viso_amd/csrc/{f}"], capture_output=True,
                             text=True, cwd=ROOT).stdout
        with tempfile.NamedTemporaryFile("w", suffix=".hip", dir=CSRC, delete=False) as t:
            t.write(src)
        try:
            print(f"--- {sys.argv[2]}")
            show(usage(t.name))
        finally:
            os.unlink(t.name)
