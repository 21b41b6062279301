"""Synthetic SRN-format data.

The SRN cars/chairs blobs are not shipped with the reference
(`.MISSING_LARGE_BLOBS:1-2`) and there is no network, so:

* :func:`write_synthetic_srn` writes a miniature SRN tree (RGBA PNGs, 4x4
  cam-to-world poses on an orbit looking at the origin, SRN-style 3x3
  intrinsics) plus the reference-format index pickle and a JSON twin -- used by
  the dataset / loader / CLI tests;
* :class:`SyntheticBatches` produces SRN-shaped training batches directly on
  the device (benchmarks: BASELINE.json "synthetic data"), so the timed region
  measures the training step, not PNG decoding.
"""
from __future__ import annotations

import json
import math
import os
import pickle
from typing import Dict, Tuple

import numpy as np
import torch

SRN_FOCAL_128 = 131.25   # SRN cars 128^2 pinhole (fx = fy), principal point at 64
SRN_RADIUS = 1.3


def look_at_pose(pos: np.ndarray) -> np.ndarray:
    """OpenCV cam-to-world (x right, y down, z forward) looking at the origin."""
    fwd = -pos / np.linalg.norm(pos)
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    if np.linalg.norm(right) < 1e-6:
        right = np.array([1.0, 0.0, 0.0])
    right = right / np.linalg.norm(right)
    down = np.cross(fwd, right)
    M = np.eye(4)
    M[:3, 0], M[:3, 1], M[:3, 2], M[:3, 3] = right, down, fwd, pos
    return M


def orbit_position(rng: np.random.Generator, radius: float = SRN_RADIUS) -> np.ndarray:
    az = rng.uniform(0, 2 * math.pi)
    el = rng.uniform(0.05, 1.0)
    return radius * np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])


def _blob_image(rng: np.random.Generator, size: int) -> np.ndarray:
    yy, xx = np.mgrid[0:size, 0:size] / size
    img = np.zeros((size, size, 3))
    for _ in range(4):
        c = rng.uniform(0.2, 0.8, 2)
        s = rng.uniform(0.05, 0.25)
        col = rng.uniform(0, 1, 3)
        w = np.exp(-((xx - c[0]) ** 2 + (yy - c[1]) ** 2) / (2 * s * s))
        img += w[..., None] * col
    return np.clip(img, 0, 1)


def write_synthetic_srn(root: str, num_instances: int = 10, num_views: int = 6, size: int = 128,
                        seed: int = 0) -> Dict[str, list]:
    """Write ``root/<id>/{rgb,pose,intrinsics}`` + ``root/index.pkl|.json``."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    index = {}
    f = SRN_FOCAL_128 * size / 128.0
    K = np.array([[f, 0, size / 2], [0, f, size / 2], [0, 0, 1.0]])
    for i in range(num_instances):
        inst = f"{i:06x}{rng.integers(0, 1 << 30):08x}"
        for sub in ("rgb", "pose", "intrinsics"):
            os.makedirs(os.path.join(root, inst, sub), exist_ok=True)
        views = []
        for v in range(num_views):
            name = f"{v:06d}.png"
            rgb = (_blob_image(rng, size) * 255).astype(np.uint8)
            rgba = np.concatenate([rgb, np.full((size, size, 1), 255, np.uint8)], -1)
            Image.fromarray(rgba, "RGBA").save(os.path.join(root, inst, "rgb", name))
            pose = look_at_pose(orbit_position(rng))
            np.savetxt(os.path.join(root, inst, "pose", name[:-4] + ".txt"), pose.reshape(1, 16), fmt="%.8f")
            np.savetxt(os.path.join(root, inst, "intrinsics", name[:-4] + ".txt"), K.reshape(1, 9), fmt="%.6f")
            views.append(name)
        index[inst] = views
    with open(os.path.join(root, "index.pkl"), "wb") as fh:
        pickle.dump(index, fh)
    with open(os.path.join(root, "index.json"), "w") as fh:
        json.dump(index, fh)
    return index


def random_orbit_poses(n: int, generator: torch.Generator, device, radius: float = SRN_RADIUS
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Batched look-at cam-to-world poses (float64): R [n,3,3], t [n,3]."""
    az = torch.rand(n, generator=generator, device=device, dtype=torch.float64) * 2 * math.pi
    el = 0.05 + torch.rand(n, generator=generator, device=device, dtype=torch.float64) * 0.95
    pos = radius * torch.stack([torch.cos(el) * torch.cos(az), torch.cos(el) * torch.sin(az), torch.sin(el)], -1)
    fwd = -pos / pos.norm(dim=-1, keepdim=True)
    up = torch.tensor([0.0, 0.0, 1.0], dtype=torch.float64, device=device).expand_as(fwd)
    right = torch.linalg.cross(fwd, up)
    right = right / right.norm(dim=-1, keepdim=True)
    down = torch.linalg.cross(fwd, right)
    R = torch.stack([right, down, fwd], dim=-1)
    return R, pos


class SyntheticBatches:
    """Infinite iterator of on-device SRN-shaped batches
    ``(img[B,2,3,H,W] f32 in [-1,1], R[B,2,3,3] f64, T[B,2,3] f64, K[B,3,3] f64)``."""

    def __init__(self, batch_size: int, imgsize: int = 64, device="cpu", seed: int = 0,
                 focal_ref_size: int = 128):
        self.B, self.S = batch_size, imgsize
        self.device = torch.device(device)
        self.g = torch.Generator(device=self.device)
        self.g.manual_seed(seed)
        # SRN K at its native 128^2 (D10: not rescaled to imgsize)
        f = SRN_FOCAL_128 * focal_ref_size / 128.0
        c = focal_ref_size / 2.0
        self.K = torch.tensor([[f, 0, c], [0, f, c], [0, 0, 1.0]], dtype=torch.float64, device=self.device)

    def __iter__(self):
        return self

    def __next__(self):
        B, S = self.B, self.S
        low = torch.rand(B * 2, 3, 8, 8, generator=self.g, device=self.device) * 2 - 1
        img = torch.nn.functional.interpolate(low, size=(S, S), mode="bilinear", align_corners=False)
        img = img.reshape(B, 2, 3, S, S).clamp(-1, 1)
        R, t = random_orbit_poses(B * 2, self.g, self.device)
        return img, R.reshape(B, 2, 3, 3), t.reshape(B, 2, 3), self.K.expand(B, 3, 3).contiguous()
