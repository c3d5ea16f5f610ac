"""Device ops backed by the gfx950 kernels in ``csrc/kernels/kernels.hip``."""
from .colsum import colsum
from .reduce import chunk_reduce, count_expand

__all__ = ["chunk_reduce", "colsum", "count_expand"]
