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
        # low-precision copy of pflat kept current by the fused update (use_shadow)
        self.sflat: Optional[torch.Tensor] = None
        self._shadow_on = False
        self._shadow_versions: Optional[List[int]] = None
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

    # ---- bf16 shadow weights -------------------------------------------------
    # A bf16 forward under autocast casts every fp32 weight to bf16 each step
    # (4 B read + 2 B written per parameter).  With flattened fp32 parameters
    # the fused average + SGD pass (``count_mean`` kernel) can store the bf16
    # copy of each updated parameter as it writes it, so the next forward reads
    # that copy instead: the cast disappears from the step.
    #
    # The shadow is trusted only while nothing else touched the parameters: a
    # torch in-place op on a parameter bumps its version counter, and any
    # mismatch with the versions recorded at the last refresh re-copies the
    # shadow (our kernel writes through raw pointers and bumps none).  Writes
    # through ``p.data`` bypass the counter (torch's documented caveat): call
    # ``invalidate_shadow()`` after such writes.

    def use_shadow(self, dtype: Optional[torch.dtype]) -> bool:
        """Keep a ``dtype`` copy of the parameters current from now on (None:
        stop updating it).  Returns whether the shadow is in use."""
        ok = (dtype is not None and dtype != self.flat.dtype and self.pflat is not None
              and self.pflat.is_cuda and self.pflat.dtype == torch.float32 and dtype == torch.bfloat16
              and self.params_bound())
        if not ok:
            self._shadow_on = False
            return False
        if self.sflat is None or self.sflat.dtype != dtype:
            self.sflat = torch.empty(self.numel, dtype=dtype, device=self.pflat.device)
            self._shadow_versions = None
        if not self._shadow_on or self._shadow_versions != [p._version for p in self.params]:
            self.sflat.copy_(self.pflat)
            self._shadow_versions = [p._version for p in self.params]
        self._shadow_on = True
        return True

    def invalidate_shadow(self) -> None:
        self._shadow_versions = None

    def shadow_of(self, p: torch.nn.Parameter) -> Optional[torch.Tensor]:
        """The current low-precision copy of parameter ``p`` (None if the
        shadow is not in use)."""
        if not self._shadow_on or self.sflat is None:
            return None
        off = 0
        for q in self.params:
            if q is p:
                return self.sflat[off:off + p.numel()].view_as(p)
            off += q.numel()
        return None

    def params_bound(self) -> bool:
        """Is every parameter still its view of ``pflat``?"""
        if self.pflat is None:
            return False
        off = 0
        es = self.pflat.element_size()
        base = self.pflat.data_ptr()
        for p in self.params:
            if p.data_ptr() != base + off * es:
                return False
            off += p.numel()
        return True

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


    def sgd_from(self, allreduce: Optional[AllreduceFn], lr: float,
                 out_buf: Optional[torch.Tensor] = None) -> Optional[AllReduceOutput]:
        """Average the gradients over the contributors and apply SGD.  With
        flattened parameters this is one fused pass over the allreduce output
        (no averaged-gradient tensor is written).  ``out_buf``: the round's
        output buffer (reused; a captured step needs fixed buffers)."""
        if allreduce is None:
            sgd_step(self.params, lr)
            return None
        out = allreduce(self.flat) if out_buf is None else allreduce(self.flat, out=out_buf)
        if self.pflat is not None and out.data.dtype == self.pflat.dtype:
            out.axpy_mean_(self.pflat, -lr, shadow=self.sflat if self._shadow_on else None)
        else:
            self.average_out(out)
            sgd_step(self.params, lr)
            if self._shadow_on and self.sflat is not None:
                self.sflat.copy_(self.pflat)
        if self._shadow_on:
            # versions after our own update (sgd_step's in-place adds bump them)
            self._shadow_versions = [p._version for p in self.params]
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
