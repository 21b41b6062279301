"""SRN cars/chairs dataset (reference: `SRNdataset.py:12-95`).

Contract kept from the reference:
  * ``<root>/<instance>/rgb/<view>.png``, ``pose/<view>.txt`` (16 floats,
    cam-to-world 4x4), ``intrinsics/<view>.txt`` (9 floats, 3x3 K);
  * index ``{instance_id: [view png names]}`` (the reference's ``cars.pickle``);
  * split: ``sorted`` ids shuffled with ``random.seed(0)``, first 90 % train,
    rest val (`SRNdataset.py:50-57`);
  * item: 2 distinct random views -> ``imgs[2,3,H,W] f32 in [-1,1]`` (alpha
    dropped), ``R[2,3,3] f64``, ``T[2,3] f64``, ``K[3,3] f64`` taken from the
    instance's first view and NOT rescaled with imgsize (D10).

Differences by design: the pair draw uses a per-(epoch, index) RNG (the
reference uses the process-global ``random`` module, so pairs differ per
worker).  The epoch travels WITH each index: :class:`ShardSampler` (``with_epoch``)
yields ``(epoch, idx)`` keys, so persistent DataLoader workers -- which hold
their own copy of the dataset and never see ``set_epoch`` on the main
process's copy -- still draw a fresh view pair every epoch.  The index may
also be JSON or discovered by scanning, and pickled
indices are read with a restricted unpickler that only admits plain
containers of strings (no code execution).
"""
from __future__ import annotations

import io
import json
import os
import pickle
import random
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, Sampler


class _SafeUnpickler(pickle.Unpickler):
    """Only builtins containers/str/int/float are allowed; any global lookup
    (class / function reference) is refused."""

    def find_class(self, module, name):  # pragma: no cover - exercised by malicious input only
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from index pickle")


def load_index(index_path: str) -> Dict[str, List[str]]:
    if index_path.endswith(".json"):
        with open(index_path) as f:
            d = json.load(f)
    else:
        with open(index_path, "rb") as f:
            d = _SafeUnpickler(io.BytesIO(f.read())).load()
    if not isinstance(d, dict):
        raise ValueError(f"index {index_path} is not a dict")
    return {str(k): [str(v) for v in vs] for k, vs in d.items()}


def scan_index(root: str) -> Dict[str, List[str]]:
    out = {}
    for inst in sorted(os.listdir(root)):
        rgb = os.path.join(root, inst, "rgb")
        if os.path.isdir(rgb):
            views = sorted(v for v in os.listdir(rgb) if v.endswith(".png"))
            if len(views) >= 2:
                out[inst] = views
    return out


def split_ids(ids: Sequence[str], split: str) -> List[str]:
    allv = sorted(ids)
    random.Random(0).shuffle(allv)
    n = int(len(allv) * 0.9)
    return allv[:n] if split == "train" else allv[n:]


def read_matrix(path: str, shape) -> np.ndarray:
    with open(path) as f:
        vals = np.array(f.read().strip().split()).astype(np.float64)
    return vals[: int(np.prod(shape))].reshape(shape)


def load_image(path: str, imgsize: int) -> np.ndarray:
    from PIL import Image
    img = Image.open(path)
    if imgsize != img.size[0] or imgsize != img.size[1]:
        img = img.resize((imgsize, imgsize))
    arr = np.asarray(img, dtype=np.float64) / 255.0 * 2.0 - 1.0
    if arr.ndim == 2:
        arr = np.stack([arr] * 3, -1)
    return arr.transpose(2, 0, 1)[:3].astype(np.float32)


def split_key(key, default_epoch: int):
    """Dataset key -> (epoch, index): ``(epoch, idx)`` from an epoch-carrying
    sampler, or a plain index drawn under the dataset's own epoch."""
    if isinstance(key, (tuple, list)):
        return int(key[0]), int(key[1])
    return default_epoch, int(key)


class SRNDataset(Dataset):
    """``SRNDataset(split, path, index, imgsize)`` -> (imgs, R, T, K)."""

    def __init__(self, split: str = "train", path: str = "./data/SRN/cars_train", index: str = "",
                 imgsize: int = 128, seed: int = 0):
        super().__init__()
        self.path = path
        self.imgsize = imgsize
        self.seed = seed
        self.epoch = 0
        if index and os.path.exists(index):
            self.index = load_index(index)
        else:
            self.index = scan_index(path)
        self.ids = split_ids(list(self.index.keys()), split)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __len__(self) -> int:
        return len(self.ids)

    def __getitem__(self, key):
        epoch, idx = split_key(key, self.epoch)
        inst = self.ids[idx]
        views = self.index[inst]
        K = read_matrix(os.path.join(self.path, inst, "intrinsics", views[0][:-4] + ".txt"), (3, 3))
        rng = random.Random((self.seed * 1000003 + epoch) * 1000003 + idx)
        pair = rng.sample(views, 2)
        imgs, poses = [], []
        for v in pair:
            imgs.append(load_image(os.path.join(self.path, inst, "rgb", v), self.imgsize))
            poses.append(read_matrix(os.path.join(self.path, inst, "pose", v[:-4] + ".txt"), (4, 4)))
        imgs = np.stack(imgs, 0)
        poses = np.stack(poses, 0)
        return imgs, poses[:, :3, :3], poses[:, :3, 3], K


class ShardSampler(Sampler):
    """DistributedSampler-equivalent (fixes D1: the reference passes the
    sampler *as the dataset*).  Shuffles with (seed, epoch), pads to a multiple
    of world size, returns this rank's strided shard.  ``with_epoch``: yield
    ``(epoch, idx)`` keys so the dataset's pair draw follows the epoch even
    inside persistent worker processes."""

    def __init__(self, n: int, rank: int = 0, world: int = 1, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False, with_epoch: bool = False):
        self.n, self.rank, self.world = n, rank, world
        self.with_epoch = with_epoch
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        self.start = 0
        if drop_last:
            self.num = n // world
        else:
            self.num = (n + world - 1) // world
        self.total = self.num * world

    def set_epoch(self, epoch: int, start: int = 0) -> None:
        """``start``: skip this rank's first ``start`` indices of the epoch
        (mid-epoch resume continues where the checkpoint left off)."""
        self.epoch = epoch
        self.start = max(0, min(int(start), self.num))

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if self.total > len(idx):
            idx = idx + idx[: self.total - len(idx)]
        idx = idx[: self.total]
        mine = idx[self.rank: self.total: self.world][self.start:]
        if self.with_epoch:
            return iter([(self.epoch, i) for i in mine])
        return iter(mine)

    def __len__(self) -> int:
        return self.num - self.start


def collate(items):
    imgs, R, T, K = zip(*items)
    return (torch.from_numpy(np.stack(imgs)), torch.from_numpy(np.stack(R)),
            torch.from_numpy(np.stack(T)), torch.from_numpy(np.stack(K)))


class MultiEpochsDataLoader(DataLoader):
    """Persistent-worker loader (reference `SRNdataset.py:12-40` swaps in an
    infinite batch sampler to keep workers alive; ``persistent_workers`` does
    the same natively)."""

    def __init__(self, dataset, batch_size: int, sampler=None, shuffle: bool = False, num_workers: int = 0,
                 drop_last: bool = True, pin_memory: bool = False):
        kw = {}
        if num_workers > 0:
            kw.update(persistent_workers=True, prefetch_factor=4)
        super().__init__(dataset, batch_size=batch_size, sampler=sampler,
                         shuffle=shuffle if sampler is None else False, num_workers=num_workers,
                         drop_last=drop_last, collate_fn=collate, pin_memory=pin_memory, **kw)
