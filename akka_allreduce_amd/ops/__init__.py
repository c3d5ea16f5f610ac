"""Device ops backed by the gfx950 kernels in ``csrc/kernels/kernels.hip``."""
from .colsum import colsum
from .reduce import chunk_reduce, count_expand
from .xent import cross_entropy

__all__ = ["chunk_reduce", "colsum", "count_expand", "cross_entropy"]
