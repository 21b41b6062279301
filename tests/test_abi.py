"""Every C ABI entry point declared in ops/_abi.py is exported by the built
gfx950 library (catches a kernel file edit that dropped a symbol before the
GPU box does).  Skipped when the library has not been built here."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed_3d_diffusion_pytorch_amd", "ops", "libd3d_hip.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_abi_symbols_exported():
    src = open(os.path.join(ROOT, "distributed_3d_diffusion_pytorch_amd", "ops", "_abi.py")).read()
    names = re.findall(r'"(d3d_\w+)"', src)
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in syms]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_no_unresolved_kernel_stubs():
    """A kernel whose host stub was not emitted (e.g. device-only types in a
    host-visible lambda) links fine but fails at dlopen on the GPU box."""
    out = subprocess.check_output(["nm", "-u", LIB]).decode()
    bad = [line for line in out.splitlines() if "__device_stub__" in line]
    assert not bad, bad
