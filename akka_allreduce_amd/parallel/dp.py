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
    """``flatten_params=True`` also moves the parameters into one flat buffer
    with the gradients' layout, so the SGD update fuses into the averaging
    (``sgd_from``: one pass ``p -= lr * sum / count`` on the GPU)."""

    def __init__(self, params: List[torch.nn.Parameter], dtype: Optional[torch.dtype] = None,
                 flatten_params: bool = False):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        dt = dtype or self.params[0].dtype
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=dt, device=dev)
        self.pflat: Optional[torch.Tensor] = None
        if flatten_params and all(p.dtype == dt for p in self.params):
            self.pflat = torch.empty(self.numel, dtype=dt, device=dev)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            if self.pflat is not None:
                view = self.pflat[off:off + n].view_as(p)
                view.copy_(p.data)
                p.data = view
            off += n

    def zero_(self) -> None:
        self.flat.zero_()

    def bound(self) -> bool:
        """Is every parameter's ``.grad`` still its view of ``flat``?"""
        off = 0
        es = self.flat.element_size()
        base = self.flat.data_ptr()
        for p in self.params:
            g = p.grad
            if g is None or g.data_ptr() != base + off * es or g.shape != p.shape:
                return False
            off += p.numel()
        return True

    def rebind(self) -> bool:
        """Re-attach every ``.grad`` that is no longer a view of ``flat``
        (``zero_grad()`` sets them to ``None`` by default; an optimizer or
        user code may assign fresh tensors).  Any gradient held outside the
        bucket is copied into its view first.  Returns True if anything had
        to be re-attached."""
        if self.bound():
            return False
        off = 0
        for p in self.params:
            n = p.numel()
            view = self.flat[off:off + n].view_as(p)
            g = p.grad
            if g is None:
                view.zero_()
            elif g.data_ptr() != view.data_ptr():
                view.copy_(g)
            p.grad = view
            off += n
        return True

    def average(self, allreduce: Optional[AllreduceFn]) -> Optional[AllReduceOutput]:
        """flat <- mean over contributors (no-op without an allreduce)."""
        if allreduce is None:
            return None
        out = allreduce(self.flat)
        self.average_out(out)  # one fused pass on the GPU, straight into the bucket
        return out


    def sgd_from(self, allreduce: Optional[AllreduceFn], lr: float) -> Optional[AllReduceOutput]:
        """Average the gradients over the contributors and apply SGD.  With
        flattened parameters this is one fused pass over the allreduce output
        (no averaged-gradient tensor is written)."""
        if allreduce is None:
            sgd_step(self.params, lr)
            return None
        out = allreduce(self.flat)
        if self.pflat is not None and out.data.dtype == self.pflat.dtype:
            out.axpy_mean_(self.pflat, -lr)
        else:
            self.average_out(out)
            sgd_step(self.params, lr)
        return out

    def average_out(self, out: AllReduceOutput) -> None:
        if out.data.dtype == self.flat.dtype:
            out.mean(out=self.flat)
        else:
            self.flat.copy_(out.mean().to(self.flat.dtype))


def sgd_step(params: List[torch.nn.Parameter], lr: float) -> None:
    with torch.no_grad():
        for p in params:
            if p.grad is not None:
                p.add_(p.grad, alpha=-lr)
