"""Build the gfx950 HIP library in-tree: viso_amd/libviso_amd.so.

Every ``csrc/*.hip`` / ``csrc/*.cpp`` file is compiled by hipcc for
``--offload-arch=gfx950`` with ``-ffp-contract=off`` (the numerics contract
of DESIGN.md §Numerics) and linked into one shared library exporting the C
ABI of ``include/viso/viso_c.h``.  Objects are rebuilt only when a source or
header is newer than the object.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
# VISO_VARIANT=probe builds an instrumented copy (-DVISO_PROBE) next to the
# product library (libviso_amd_probe.so, objects in _obj_probe); the product
# path never loads it (viso_amd/_lib.py loads it only when VISO_LIB names it).
VARIANT = os.environ.get("VISO_VARIANT", "")
OBJ = os.path.join(HERE, "_obj" + (f"_{VARIANT}" if VARIANT else ""))
LIB = os.path.join(HERE, "libviso_amd" + (f"_{VARIANT}" if VARIANT else "") + ".so")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("VISO_OFFLOAD_ARCH", "gfx950")

COMMON = ["-std=c++17", "-O3", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
          "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-Wno-unused-result",
          # leading scalar kernel arguments arrive in SGPRs (direct_level_kernel's
          # prologue pointers): no kernel-argument load ahead of the first loads
          "-mllvm", "-amdgpu-kernarg-preload-count=5"]
if VARIANT == "probe":
    COMMON.append("-DVISO_PROBE")
# experiment builds (dev): extra -D flags for a variant library, e.g.
# VISO_VARIANT=lk4 VISO_DEFS="-DVISO_LK_MIN_WAVES=4"
if VARIANT and os.environ.get("VISO_DEFS"):
    COMMON.extend(os.environ["VISO_DEFS"].split())


def source_hash() -> str:
    """sha256 (first 16 hex digits) over the library's sources and public
    headers (viso_amd/csrc/*, include/viso/*, by relative path and content)
    and the build flags.  Compiled into viso_version() (-DVISO_SOURCE_HASH),
    so a prebuilt library whose sources changed since its build is detected
    (viso_amd._lib.check_source_hash, __graft_entry__.smoke)."""
    import hashlib
    h = hashlib.sha256()
    for d in (CSRC, os.path.join(ROOT, "include", "viso")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".cpp", ".hpp", ".h")):
                h.update(os.path.relpath(os.path.join(d, f), ROOT).encode())
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    # the flags, with the tree's location taken out (the GPU box runs a copy
    # of the tree under another path)
    h.update(" ".join(COMMON).replace(ROOT, "<root>").encode())
    return h.hexdigest()[:16]


def _headers():
    hs = []
    for d in (CSRC, os.path.join(ROOT, "include", "viso")):
        for f in os.listdir(d):
            if f.endswith((".hpp", ".h")):
                hs.append(os.path.join(d, f))
    return hs


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                  if f.endswith((".hip", ".cpp")))


def _compile(src, hdr_mtime, verbose, shash):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    # context.hip carries the source hash (viso_version): rebuilt whenever the
    # hash its object was built with differs
    versioned = os.path.basename(src) == "context.hip"
    stamp = obj + ".hash"
    fresh = os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime)
    if versioned and fresh:
        fresh = os.path.exists(stamp) and open(stamp).read().strip() == shash
    if fresh:
        return obj
    flags = [*COMMON, f'-DVISO_SOURCE_HASH="{shash}"'] if versioned else COMMON
    cmd = [HIPCC, *flags, "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, *flags, "-x", "hip", "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"hipcc failed on {src}")
    if versioned:
        with open(stamp, "w") as fh:
            fh.write(shash)
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    hdr_mtime = max([os.path.getmtime(h) for h in _headers()] + [0.0])
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    shash = source_hash()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr_mtime, verbose, shash), srcs))
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(o) for o in objs):
        return LIB
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs, "-lpthread", "-lz", "-lrocprofiler-sdk-roctx"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("link failed")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
