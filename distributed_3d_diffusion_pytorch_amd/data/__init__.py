from .srn import SRNDataset, ShardSampler, MultiEpochsDataLoader, collate, load_index, scan_index, split_ids
from .cache import CachedSRNDataset, build_cache
from .fastloader import CachedBatchLoader
from .synthetic import SyntheticBatches, write_synthetic_srn, look_at_pose, random_orbit_poses

# reference-compatible alias (`SRNdataset.py:42`)
dataset = SRNDataset

__all__ = ["CachedBatchLoader", "CachedSRNDataset", "build_cache", "SRNDataset", "dataset", "ShardSampler", "MultiEpochsDataLoader", "collate", "load_index",
           "scan_index", "split_ids", "SyntheticBatches", "write_synthetic_srn", "look_at_pose",
           "random_orbit_poses"]
