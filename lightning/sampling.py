#!/usr/bin/env python
"""Sampling CLI of the Lightning variant (reference `lightning/sampling.py`):
the root sampler with the reference's ``./../`` default paths (`:21-22`), for
running from inside ``lightning/``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import sampling as _root_sampling  # noqa: E402


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not any(a == "--model" or a.startswith("--model=") for a in argv):
        argv += ["--model", "./../trained_model.pt"]
    if not any(a == "--target" or a.startswith("--target=") for a in argv):
        argv += ["--target", "./../data/SRN/cars_train/a4d535e1b1d3c153ff23af07d9064736"]
    _root_sampling.main(argv)


if __name__ == "__main__":
    main()
