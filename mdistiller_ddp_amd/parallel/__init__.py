"""Data-parallel layer: process-group bootstrap, flat-gradient all-reduce,
BN-buffer sync, metric reduction, CRD memory-update exchange."""
from .dist import (init_distributed, destroy, get_rank, get_world_size, get_local_rank,
                   is_dist, is_master, barrier, DistInfo)
from .grad_reducer import GradReducer
from .replicate import broadcast_initial_state, state_checksum
from . import dist_fn

__all__ = ["init_distributed", "destroy", "get_rank", "get_world_size", "get_local_rank",
           "is_dist", "is_master", "barrier", "DistInfo", "GradReducer", "dist_fn",
           "broadcast_initial_state", "state_checksum"]
