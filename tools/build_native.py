#!/usr/bin/env python
"""Build the in-tree gfx950 HIP library ``ops/libd3d_hip.so``.

Plain ``hipcc --offload-arch=gfx950`` per translation unit (parallel), then a
shared link.  No torch headers, no hipify: the library exposes a C ABI that
``ops/_abi.py`` declares for ctypes.  Incremental: objects are rebuilt only
when their source or ``common.h`` changed.

    python tools/build_native.py [--force] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_3d_diffusion_pytorch_amd")
SRC = os.path.join(PKG, "ops", "csrc")
OUT = os.path.join(PKG, "ops", "libd3d_hip.so")
OBJ = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("D3D_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def sources():
    return sorted(os.path.join(SRC, f) for f in os.listdir(SRC) if f.endswith(".hip"))


def build(force: bool = False, jobs: int = 8, debug: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    cc = hipcc()
    hdrs = [os.path.join(SRC, f) for f in os.listdir(SRC) if f.endswith(".h")]
    hdr_mtime = max((os.path.getmtime(h) for h in hdrs), default=0)
    flags = ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
    flags += ["-O0", "-g"] if debug else ["-O3"]

    def compile_one(src: str) -> str:
        obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
            return obj
        cmd = [cc, *flags, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stderr}")
        if verbose:
            print(f"[build] {os.path.basename(src)}", flush=True)
        return obj

    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(o) for o in objs):
        cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stderr}")
        if verbose:
            print(f"[build] linked {OUT}", flush=True)
    return OUT


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    build(a.force, a.jobs, a.debug)


if __name__ == "__main__":
    sys.exit(main())
