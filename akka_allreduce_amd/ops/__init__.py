"""Device ops backed by the gfx950 kernels in ``csrc/kernels/kernels.hip``."""
from .reduce import chunk_reduce, count_expand

__all__ = ["chunk_reduce", "count_expand"]
