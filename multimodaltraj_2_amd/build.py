"""Compile libg2k_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

Each csrc/*.hip translation unit is compiled to an object in parallel, then
linked into one shared library (no device code crosses translation units)."""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRC = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
CXX_SRC = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))   # host-only C++ (g++)
HDR = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "g2k_hip.h")]
OUT = os.path.join(HERE, "libg2k_hip.so")
OBJ = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fno-slp-vectorize", "-std=c++17", "-fPIC",
         "-I" + os.path.join(ROOT, "include")]
# the scene kernel: no loop strength reduction (its per-stream induction
# registers cost more VGPRs than the address arithmetic they save; measured
# 125 -> 119 VGPRs, no spills in train mode's producers)
FILE_FLAGS = {"g2k_scene.hip": ["-mllvm", "-disable-lsr"]}


def flags_for(src):
    return FLAGS + FILE_FLAGS.get(os.path.basename(src), [])


def kernel_tree_sha() -> str:
    """sha256 over the library's sources (csrc/*.hip, *.cpp, *.h and the ABI
    header), names and bytes: identifies the kernel tree a profile was taken
    on (tools/collect_pmc.py records it, bench.py compares)."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(SRC + CXX_SRC + HDR):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SRC + CXX_SRC + HDR + [os.path.abspath(__file__)])


CXX = os.environ.get("CXX", "g++")
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-I" + os.path.join(ROOT, "include")]


def _compile(src, verbose):
    obj = os.path.join(OBJ, os.path.splitext(os.path.basename(src))[0] + ".o")
    if src.endswith(".cpp"):
        cmd = [CXX, *CXX_FLAGS, "-c", "-o", obj, src]
    else:
        cmd = [HIPCC, *flags_for(src), "-c", "-o", obj, src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return obj


def _obj_current(src) -> bool:
    """The object of `src` is newer than it, every header and this file (a
    header change rebuilds every translation unit)."""
    obj = os.path.join(OBJ, os.path.splitext(os.path.basename(src))[0] + ".o")
    if not os.path.exists(obj):
        return False
    t = os.path.getmtime(obj)
    return all(os.path.getmtime(p) <= t for p in [src] + HDR + [os.path.abspath(__file__)])


def build(force: bool = False, verbose: bool = True) -> str:
    if force or needs_build():
        os.makedirs(OBJ, exist_ok=True)
        units = SRC + CXX_SRC

        def unit(s):
            if not force and _obj_current(s):
                return os.path.join(OBJ, os.path.splitext(os.path.basename(s))[0] + ".o")
            return _compile(s, verbose)
        with ThreadPoolExecutor(max_workers=min(8, len(units))) as ex:
            objs = list(ex.map(unit, units))
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
