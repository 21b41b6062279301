"""In-process A/B wrapper around bench.py: AB_FILM_EV=0/1 (per-block FiLM GEMMs
on the conditioning stream), AB_S64=cfg (small-grid conv wave groups, 0 =
automatic, 1 = one group); remaining arguments go to bench.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributed_3d_diffusion_pytorch_amd.models import xunet as X
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H
    if "AB_FILM_EV" in os.environ:
        X.FILM_BLOCK_EVENTS = os.environ["AB_FILM_EV"] == "1"
    if "AB_S64" in os.environ:
        H._lib.d3d_conv_s64_cfg(int(os.environ["AB_S64"]))
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()


if __name__ == "__main__":
    main()
