from .checkpoint import (save_checkpoint, load_checkpoint, load_model_weights, find_resume, strip_prefix,
                         add_prefix, atomic_save)
from .metrics import MetricsLogger, StepTimer, train_flops_per_example, range_push, check_finite

__all__ = ["save_checkpoint", "load_checkpoint", "load_model_weights", "find_resume", "strip_prefix",
           "add_prefix", "atomic_save", "MetricsLogger", "StepTimer", "train_flops_per_example", "range_push",
           "check_finite"]
