import os
import pickle

import numpy as np
import pytest
import torch

from distributed_3d_diffusion_pytorch_amd.data import (SRNDataset, ShardSampler, MultiEpochsDataLoader,
                                                       write_synthetic_srn, load_index, split_ids)


@pytest.fixture(scope="module")
def srn_root(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("srn"))
    write_synthetic_srn(root, num_instances=10, num_views=5, size=32, seed=0)
    return root


def test_split_is_reference_deterministic(srn_root):
    idx = load_index(os.path.join(srn_root, "index.pkl"))
    tr, va = split_ids(list(idx), "train"), split_ids(list(idx), "val")
    assert len(tr) == 9 and len(va) == 1 and not set(tr) & set(va)
    import random
    allv = sorted(idx)
    random.seed(0)
    random.shuffle(allv)
    assert tr == allv[:9]                  # SRNdataset.py:50-57


def test_item(srn_root):
    ds = SRNDataset("train", srn_root, os.path.join(srn_root, "index.json"), imgsize=16)
    imgs, R, T, K = ds[0]
    assert imgs.shape == (2, 3, 16, 16) and imgs.dtype == np.float32
    assert imgs.min() >= -1 and imgs.max() <= 1
    assert R.shape == (2, 3, 3) and T.shape == (2, 3) and K.shape == (3, 3)
    assert abs(K[0, 0] - 131.25 * 32 / 128) < 1e-4       # K not rescaled to imgsize (D10)
    assert np.allclose(R[0] @ R[0].T, np.eye(3), atol=1e-6)


def test_scan_index_matches_pickle(srn_root):
    a = SRNDataset("train", srn_root, "", imgsize=16)
    b = SRNDataset("train", srn_root, os.path.join(srn_root, "index.pkl"), imgsize=16)
    assert a.ids == b.ids


def test_safe_unpickler_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    p = tmp_path / "evil.pkl"
    p.write_bytes(pickle.dumps({"x": Evil()}))
    with pytest.raises(pickle.UnpicklingError):
        load_index(str(p))


def test_shard_sampler_disjoint_covering():
    n, world = 23, 4
    shards = []
    for r in range(world):
        s = ShardSampler(n, r, world, shuffle=True, seed=3)
        s.set_epoch(2)
        shards.append(list(s))
    assert all(len(x) == len(shards[0]) for x in shards)
    allidx = sum(shards, [])
    assert set(allidx) == set(range(n))
    s0 = ShardSampler(n, 0, world, seed=3)
    s0.set_epoch(1)
    assert list(s0) != shards[0]           # reshuffled per epoch


def test_loader(srn_root):
    ds = SRNDataset("train", srn_root, "", imgsize=16)
    dl = MultiEpochsDataLoader(ds, batch_size=4, sampler=ShardSampler(len(ds), 0, 1), num_workers=2)
    for _ in range(2):
        batches = list(dl)
        assert len(batches) == 2
        img, R, T, K = batches[0]
        assert img.shape == (4, 2, 3, 16, 16) and R.dtype == torch.float64 and K.shape == (4, 3, 3)


def test_persistent_workers_draw_new_pairs_each_epoch(srn_root):
    """Persistent workers hold their own dataset copy; the epoch must reach
    them through the sampler keys (pairs were frozen at epoch 0)."""
    ds = SRNDataset("train", srn_root, "", imgsize=16)
    sampler = ShardSampler(len(ds), 0, 1, shuffle=False, with_epoch=True)
    dl = MultiEpochsDataLoader(ds, batch_size=3, sampler=sampler, num_workers=2)
    seen = []
    for epoch in range(3):
        sampler.set_epoch(epoch)
        ds.set_epoch(epoch)             # main-process copy only (what the trainer does)
        seen.append(torch.cat([b[0] for b in dl]))
    assert not torch.equal(seen[0], seen[1]) and not torch.equal(seen[1], seen[2])
    # and it is the in-process draw for the same (epoch, index) key
    ref = torch.from_numpy(np.stack([ds[(1, i)][0] for i in range(seen[1].shape[0])]))
    assert torch.equal(seen[1], ref)


def test_cached_batch_loader_matches_dataset_and_feeds_fast(tmp_path):
    """Batch loader over the uint8 mmap cache: identical items to
    CachedSRNDataset for the same (epoch, index) keys; throughput far above
    the per-GPU consumption (~500 pairs/s at 16 per GPU)."""
    import time
    from distributed_3d_diffusion_pytorch_amd.data import build_cache, CachedSRNDataset, CachedBatchLoader
    root = str(tmp_path / "srn")
    write_synthetic_srn(root, num_instances=40, num_views=6, size=64, seed=3)
    cache = build_cache(root, str(tmp_path / "cache"), 64)
    ds = CachedSRNDataset("train", cache, seed=1)
    sampler = ShardSampler(len(ds), 0, 1, shuffle=True, seed=2, with_epoch=True)
    sampler.set_epoch(3)
    dl = CachedBatchLoader(ds, 8, sampler, "cpu")
    keys = list(sampler)
    got = list(dl)
    assert len(got) == len(dl) == len(keys) // 8
    for bi, (img, R, T, K) in enumerate(got):
        assert img.shape == (8, 2, 3, 64, 64) and img.dtype == torch.float32
        for j in range(8):
            ref = ds[keys[bi * 8 + j]]
            assert np.allclose(img[j].numpy(), ref[0], atol=1e-6)
            assert np.allclose(R[j].numpy(), ref[1]) and np.allclose(T[j].numpy(), ref[2])
            assert np.allclose(K[j].numpy(), ref[3])
    # host-side gather rate (what one rank's producer thread sustains)
    big = [(0, i % len(ds)) for i in range(4096)]
    t0 = time.perf_counter()
    for i in range(0, len(big), 16):
        dl.gather(big[i:i + 16])
    rate = len(big) / (time.perf_counter() - t0)
    print(f"cached batch gather: {rate:.0f} pairs/s")
    assert rate > 4000, rate


def test_cached_batch_loader_early_stop_releases_producer(tmp_path):
    """A consumer that stops after one batch (steps_per_epoch, max_steps, an
    exception in the step) must not leave the producer thread blocked on the
    full prefetch queue holding pinned batches."""
    import threading
    from distributed_3d_diffusion_pytorch_amd.data import build_cache, CachedSRNDataset, CachedBatchLoader
    root = str(tmp_path / "srn")
    write_synthetic_srn(root, num_instances=40, num_views=6, size=16, seed=3)
    cache = build_cache(root, str(tmp_path / "cache"), 16)
    ds = CachedSRNDataset("train", cache, seed=1)
    sampler = ShardSampler(len(ds), 0, 1, shuffle=True, seed=2, with_epoch=True)
    dl = CachedBatchLoader(ds, 2, sampler, "cpu")
    base = threading.active_count()
    for _ in range(3):
        it = iter(dl)
        next(it)
        it.close()                      # the generator's finally stops and joins the producer
    assert threading.active_count() == base
