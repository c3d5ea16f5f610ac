"""Data-parallel gradient averaging on top of the threshold allreduce.

The reference is the allreduce primitive a DP trainer would call: its
``dataSource(iteration)`` / ``dataSink(sum, counts, iteration)`` pair is the
integration hook and ``count`` lets a consumer average partial (thresholded)
sums.  ``GradientBucket`` packs every parameter gradient into one
flat buffer (the grads are views into it, so there is no pack/unpack copy) and
averages with the per-element contributor counts, so a round that completed
without a straggler's contribution still yields an unbiased mean of the
gradients that did arrive.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch

from ..data import AllReduceOutput

AllreduceFn = Callable[[torch.Tensor], AllReduceOutput]


class GradientBucket:
    def __init__(self, params: List[torch.nn.Parameter], dtype: Optional[torch.dtype] = None):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        dt = dtype or self.params[0].dtype
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=dt, device=dev)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n

    def zero_(self) -> None:
        self.flat.zero_()

    def average(self, allreduce: Optional[AllreduceFn]) -> Optional[AllReduceOutput]:
        """flat <- mean over contributors (no-op without an allreduce)."""
        if allreduce is None:
            return None
        out = allreduce(self.flat)
        if out.data.dtype == self.flat.dtype:
            out.mean(out=self.flat)  # one fused pass on the GPU, straight into the bucket
        else:
            self.flat.copy_(out.mean().to(self.flat.dtype))
        return out


def sgd_step(params: List[torch.nn.Parameter], lr: float) -> None:
    with torch.no_grad():
        for p in params:
            if p.grad is not None:
                p.add_(p.grad, alpha=-lr)
