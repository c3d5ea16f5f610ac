"""Fused cross entropy for bf16 logits (the MLP's loss in BASELINE config 5).

Under bf16 autocast ``F.cross_entropy`` upcasts the logits to fp32 and runs
log_softmax + nll_loss, and the backward runs their two backward kernels and
a downcast of the gradient: six small launches, ~40 µs per step on MI355X
(``profiles/r03/pass_n/cfg5_bf16_kernel_stats.csv``).  ``xent_fwd_kernel``
computes every row's log-sum-exp and loss in one launch (the mean over rows
combined by the last workgroup), ``xent_bwd_kernel`` writes the bf16
gradient ``(softmax - onehot) * go / n_valid`` in one more.  Label -100 is
ignored like torch's default ``ignore_index`` (mean over the rest); any other
label outside ``[0, C)`` -- an error in torch -- makes the loss NaN and is
counted on the device (``last_bad_labels()``; ``AKKA_CHECK_LABELS=1`` raises
at once, at the cost of a host synchronisation per call).

CUDA bf16 inputs always go to the native kernels (a missing extension
raises); anything else uses ``F.cross_entropy``, which is also the
numerics reference of the GPU test.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from .._native_loader import load as _load

_TICKETS: Dict[Tuple[int, int], torch.Tensor] = {}
_CHECK_LABELS = os.environ.get("AKKA_CHECK_LABELS") == "1"
_LAST: Dict[int, torch.Tensor] = {}


def last_bad_labels() -> int:
    """Targets outside ``[0, C)`` (other than -100) in the last fused call
    (synchronises); 0 before any fused call."""
    out = _LAST.get(0)
    return int(out[2].item()) if out is not None else 0


def _ticket(dev: torch.device, stream: int) -> torch.Tensor:
    key = (dev.index or 0, stream)
    t = _TICKETS.get(key)
    if t is None:  # zeroed once; every launch leaves it zero again (one per stream)
        t = torch.zeros(1, dtype=torch.int32, device=dev)
        _TICKETS[key] = t
    return t


class _FusedXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits: torch.Tensor, target: torch.Tensor):
        x = logits.contiguous()
        y = target.contiguous().to(torch.int64)
        B, C = x.shape
        stream = torch.cuda.current_stream(x.device).cuda_stream
        lse = torch.empty(B, dtype=torch.float32, device=x.device)
        rowloss = torch.empty(2 * B, dtype=torch.float32, device=x.device)
        out = torch.empty(3, dtype=torch.float32, device=x.device)  # [loss, n_valid, n_bad_labels]
        _load().xent_fwd(x.data_ptr(), y.data_ptr(), B, C, lse.data_ptr(), rowloss.data_ptr(), out.data_ptr(),
                         _ticket(x.device, stream).data_ptr(), stream)
        ctx.save_for_backward(x, y, lse, out)
        if _CHECK_LABELS and float(out[2].item()) > 0:
            raise ValueError(f"cross_entropy: {int(out[2].item())} target(s) outside [0, {C}) "
                             "(only -100 is ignored)")
        _LAST[0] = out  # last_bad_labels()
        return out[0]

    @staticmethod
    def backward(ctx, go: torch.Tensor):
        x, y, lse, out = ctx.saved_tensors
        B, C = x.shape
        g = go.to(torch.float32).contiguous()
        gx = torch.empty_like(x)
        _load().xent_bwd(x.data_ptr(), y.data_ptr(), B, C, lse.data_ptr(), out.data_ptr(), g.data_ptr(),
                         gx.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)
        return gx, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean cross entropy of ``logits`` [B, C] against class indices
    ``target`` [B]; the fused gfx950 path for CUDA bf16 logits."""
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2 and target.dim() == 1
            and target.shape[0] == logits.shape[0] and logits.shape[0] > 0):
        return _FusedXent.apply(logits, target)
    return F.cross_entropy(logits, target)
