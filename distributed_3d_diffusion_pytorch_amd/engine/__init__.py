from .optim import FusedAdam, ema_decay_for, warmup_lr
from .trainer import Trainer
from .sampler import DiffusionSampler, RecordEntry, shard_range

__all__ = ["FusedAdam", "ema_decay_for", "warmup_lr", "Trainer", "DiffusionSampler", "RecordEntry",
           "shard_range"]
