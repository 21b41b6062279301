#!/usr/bin/env python
"""Convert an SRN tree into the memory-mapped training cache
(distributed_3d_diffusion_pytorch_amd/data/cache.py)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_3d_diffusion_pytorch_amd.data.cache import build_cache  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--imgsize", type=int, default=64)
    ap.add_argument("--index", default="")
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args()
    print(build_cache(a.data, a.out, a.imgsize, a.index, a.workers))
