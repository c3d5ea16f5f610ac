"""Example models that consume the allreduce (DP-SGD)."""
from .mlp import MLP, dp_sgd_step, synthetic_batch

__all__ = ["MLP", "dp_sgd_step", "synthetic_batch"]
