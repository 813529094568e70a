"""Build libvclip.so (all HIP kernels + the C-ABI) for gfx950 with hipcc, in-tree.

The library is linked against the HIP runtime that PyTorch-ROCm itself loads
(torch/lib/libamdhip64.so, SONAME libamdhip64.so.7) via an rpath, so that a process
holding torch has exactly one HIP runtime and torch's hipStream_t values are valid
inside libvclip.  Sources are recompiled only when newer than the library.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB_PATH = os.path.join(PKG_DIR, "libvclip.so")
ARCH = os.environ.get("VCLIP_ARCH", "gfx950")
# extra hipcc flags per source file (none today)
PER_FILE_FLAGS: dict = {}


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libvclip.so)")


def _torch_libdir():
    try:
        import torch
        return os.path.join(os.path.dirname(torch.__file__), "lib")
    except Exception:
        return None


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def source_hash() -> str:
    """16-hex digest of every source libvclip.so is built from (kernels, headers, the C-ABI):
    bench.py stamps it on its JSON line and only cites profiles/ summaries of the same build."""
    import hashlib
    h = hashlib.sha256()
    deps = sources() + sorted(glob.glob(os.path.join(CSRC, "*.hpp"))) + sorted(glob.glob(os.path.join(INCLUDE, "*.h")))
    for d in deps:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB_PATH
    hipcc = _hipcc()
    objdir = os.path.join(PKG_DIR, "build")
    os.makedirs(objdir, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
              "-Wno-unused-result", "-munsafe-fp-atomics"]
    objs = []
    procs = []
    for src in sources():
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        cmd = [hipcc, *common, *PER_FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
        objs.append(obj)
    errs = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            errs.append(f"--- {src}\n{out}")
        elif verbose and out.strip():
            print(out)
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB_PATH + ".tmp", *objs]
    tl = _torch_libdir()
    if tl and os.path.exists(os.path.join(tl, "libamdhip64.so")):
        link += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
