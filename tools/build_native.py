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


def sources(src: str = SRC):
    return sorted(os.path.join(src, f) for f in os.listdir(src) if f.endswith(".hip"))


def build(force: bool = False, jobs: int = 8, debug: bool = False, verbose: bool = True, src: str = SRC,
          out: str = OUT, obj: str = OBJ) -> str:
    """``src`` / ``out`` / ``obj``: build another source tree (e.g. an older
    revision for an in-process A/B, loaded through D3D_LIB_PATH) elsewhere."""
    SRC_, OUT_, OBJ_ = src, out, obj
    os.makedirs(OBJ_, exist_ok=True)
    cc = hipcc()
    def dep_mtime(path: str, seen=None) -> float:
        """Newest mtime of a source and the local headers it includes (recursively)."""
        seen = set() if seen is None else seen
        if path in seen or not os.path.exists(path):
            return 0.0
        seen.add(path)
        t = os.path.getmtime(path)
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line.startswith("#include \""):
                    t = max(t, dep_mtime(os.path.join(os.path.dirname(path), line.split('"')[1]), seen))
        return t
    flags = ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
    flags += ["-O0", "-g"] if debug else ["-O3"]
    flags += os.environ.get("D3D_EXTRA_FLAGS", "").split()      # A/B builds (e.g. -DD3D_SIGMOID_IEEE)

    def compile_one(src: str) -> str:
        obj = os.path.join(OBJ_, os.path.basename(src)[:-4] + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= dep_mtime(src):
            return obj
        cmd = [cc, *flags, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stderr}")
        if verbose:
            print(f"[build] {os.path.basename(src)}", flush=True)
        return obj

    srcs = sources(SRC_)
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or not os.path.exists(OUT_) or os.path.getmtime(OUT_) < max(os.path.getmtime(o) for o in objs):
        cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT_]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stderr}")
        if verbose:
            print(f"[build] linked {OUT_}", flush=True)
        # a kernel whose host pass silently failed (e.g. a buffer-resource value
        # in a lambda) leaves its launch stub undefined: the library would only
        # fail to load on the GPU box
        nm = shutil.which("nm")
        if nm:
            r = subprocess.run([nm, "-D", "--undefined-only", OUT_], capture_output=True, text=True)
            bad = [l.split()[-1] for l in r.stdout.splitlines() if "__device_stub__" in l]
            if bad:
                os.remove(OUT_)
                raise RuntimeError(f"undefined kernel launch stubs in {OUT_}: {bad}")
    return OUT_


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--rev", default="", help="build ops/csrc as of this git revision into build/ab/<rev>/ "
                                              "(load it with D3D_LIB_PATH for an in-process A/B)")
    ap.add_argument("--variant", default="", help="build the CURRENT sources (with D3D_EXTRA_FLAGS) into "
                                                  "ablib/<name>/libd3d_hip.so for a same-box A/B (D3D_LIB_PATH)")
    a = ap.parse_args()
    if a.variant:
        d = os.path.join(ROOT, "ablib", a.variant)
        os.makedirs(d, exist_ok=True)
        print(build(a.force, a.jobs, a.debug, out=os.path.join(d, "libd3d_hip.so"),
                    obj=os.path.join(ROOT, "build", "ab", "variant_" + a.variant)))
        return
    if a.rev:
        d = os.path.join(ROOT, "build", "ab", a.rev)
        src = os.path.join(d, "csrc")
        os.makedirs(src, exist_ok=True)
        rel = os.path.relpath(SRC, ROOT)
        files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", f"{a.rev}:{rel}"], check=True,
                               capture_output=True, text=True).stdout.split()
        for f in files:
            blob = subprocess.run(["git", "-C", ROOT, "show", f"{a.rev}:{rel}/{f}"], check=True,
                                  capture_output=True).stdout
            with open(os.path.join(src, f), "wb") as fh:
                fh.write(blob)
        print(build(True, a.jobs, a.debug, src=src, out=os.path.join(d, "libd3d_hip.so"), obj=os.path.join(d, "obj")))
        return
    build(a.force, a.jobs, a.debug)


if __name__ == "__main__":
    sys.exit(main())
