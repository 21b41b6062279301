"""Preprocessed SRN cache: PNG decoding cannot feed thousands of examples/s
(2 PNG decodes + 3 text parses per example), so the tree is
converted ONCE into flat, memory-mappable arrays:

  images.npy  uint8 [num_instances, max_views, H, W, 3]  (resized to imgsize)
  poses.npy   float64 [num_instances, max_views, 4, 4]
  counts.npy  int32 [num_instances]                       (#views per instance)
  intrinsics.npy float64 [num_instances, 3, 3]            (first view's K, unscaled: D10)
  ids.json    instance ids in cache order

``CachedSRNDataset`` serves the same items as :class:`.srn.SRNDataset`
(identical split, pairing, normalisation) straight from ``np.load(mmap_mode='r')``
-- no decode, no text parsing, workers share the page cache.  Built with
``python tools/build_srn_cache.py --data <root> --out <dir> --imgsize 64``.
"""
from __future__ import annotations

import json
import os
import random
from typing import Dict, List, Optional

import numpy as np
from torch.utils.data import Dataset

from .srn import load_index, scan_index, split_ids, read_matrix, split_key


def build_cache(root: str, out: str, imgsize: int, index: str = "", workers: int = 8) -> str:
    from PIL import Image
    from concurrent.futures import ThreadPoolExecutor
    idx = load_index(index) if index else scan_index(root)
    ids = sorted(idx)
    V = max(len(v) for v in idx.values())
    os.makedirs(out, exist_ok=True)
    images = np.lib.format.open_memmap(os.path.join(out, "images.npy"), mode="w+", dtype=np.uint8,
                                       shape=(len(ids), V, imgsize, imgsize, 3))
    poses = np.zeros((len(ids), V, 4, 4), np.float64)
    counts = np.zeros((len(ids),), np.int32)
    Ks = np.zeros((len(ids), 3, 3), np.float64)

    def one(i):
        inst = ids[i]
        views = idx[inst]
        Ks[i] = read_matrix(os.path.join(root, inst, "intrinsics", views[0][:-4] + ".txt"), (3, 3))
        for j, v in enumerate(views):
            img = Image.open(os.path.join(root, inst, "rgb", v))
            if img.size != (imgsize, imgsize):
                img = img.resize((imgsize, imgsize))
            images[i, j] = np.asarray(img)[..., :3]
            poses[i, j] = read_matrix(os.path.join(root, inst, "pose", v[:-4] + ".txt"), (4, 4))
        counts[i] = len(views)

    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(one, range(len(ids))))
    images.flush()
    np.save(os.path.join(out, "poses.npy"), poses)
    np.save(os.path.join(out, "counts.npy"), counts)
    np.save(os.path.join(out, "intrinsics.npy"), Ks)
    with open(os.path.join(out, "ids.json"), "w") as f:
        json.dump({"ids": ids, "imgsize": imgsize}, f)
    return out


class CachedSRNDataset(Dataset):
    def __init__(self, split: str, cache_dir: str, seed: int = 0):
        with open(os.path.join(cache_dir, "ids.json")) as f:
            meta = json.load(f)
        self.all_ids: List[str] = meta["ids"]
        self.imgsize = meta["imgsize"]
        self.cache_dir = cache_dir
        pos = {k: i for i, k in enumerate(self.all_ids)}
        self.ids = split_ids(self.all_ids, split)
        self.rows = [pos[k] for k in self.ids]
        self.seed = seed
        self.epoch = 0
        self._arrs = None

    def _load(self):
        if self._arrs is None:   # opened lazily so every worker maps its own view
            d = self.cache_dir
            self._arrs = (np.load(os.path.join(d, "images.npy"), mmap_mode="r"),
                          np.load(os.path.join(d, "poses.npy")), np.load(os.path.join(d, "counts.npy")),
                          np.load(os.path.join(d, "intrinsics.npy")))
        return self._arrs

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __len__(self) -> int:
        return len(self.ids)

    def __getitem__(self, key):
        epoch, idx = split_key(key, self.epoch)
        images, poses, counts, Ks = self._load()
        r = self.rows[idx]
        rng = random.Random((self.seed * 1000003 + epoch) * 1000003 + idx)
        pair = rng.sample(range(int(counts[r])), 2)
        imgs = np.stack([images[r, j] for j in pair]).astype(np.float32) / 255.0 * 2.0 - 1.0
        imgs = imgs.transpose(0, 3, 1, 2).copy()
        P = poses[r, pair]
        return imgs, P[:, :3, :3].copy(), P[:, :3, 3].copy(), Ks[r].copy()
