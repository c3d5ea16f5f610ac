"""Distributed runtimes: SPMD/torchrun collective, master-driven cluster, simulators."""
from .collective import ThresholdAllreduce, env_rank_world, share_unique_id

__all__ = ["ThresholdAllreduce", "env_rank_world", "share_unique_id"]
