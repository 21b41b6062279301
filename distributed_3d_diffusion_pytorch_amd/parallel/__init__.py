from .dist import (DistContext, init_distributed, cleanup, spawn, barrier, get_context, all_reduce_max,
                   free_port, env_world)
from .flat import FlatParams
from .ddp import GradReducer, param_checksum, check_replicas_in_sync

__all__ = ["DistContext", "init_distributed", "cleanup", "spawn", "barrier", "get_context", "all_reduce_max",
           "free_port", "env_world", "FlatParams", "GradReducer", "param_checksum", "check_replicas_in_sync"]
