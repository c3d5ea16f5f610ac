"""Column sum of a bf16 matrix into fp32: the bias gradient of a linear layer
(``db = dY.sum(0)``) in the MLP of BASELINE config 5.

torch's generic reduction takes ~15 µs for a 256 x 8192 bf16 ``dY`` on
MI355X (``profiles/r03/pass_h/cfg5_bf16_kernel_stats.csv``): a handful of
workgroups walk all rows.  ``colsum_bf16_kernel`` (csrc/kernels/kernels.hip)
splits the rows over enough workgroups to cover the chip and combines the
fp32 partial rows deterministically in the last-arriving workgroup.

CUDA tensors always go to the native kernel (a missing extension raises);
CPU tensors use torch, which is also the numerics reference of the GPU test.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from .._native_loader import load as _load

# (device, stream, ncol, splits) -> (partials [splits, ncol] fp32, tickets [tiles] int32)
_WS: Dict[Tuple[int, int, int, int], Tuple[torch.Tensor, torch.Tensor]] = {}
_TILE = 512


def colsum(x: torch.Tensor, out: Optional[torch.Tensor] = None, splits: Optional[int] = None,
           lite: bool = True, relu_of: Optional[torch.Tensor] = None,
           masked_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out[c] = sum_r x[r, c]`` for a 2-D bf16 ``x``, fp32 result.
    ``splits`` (1..16) overrides the row split per column tile; ``lite=False``
    hands the partial rows over with fences instead of write-through stores
    (both are measurement knobs).  With ``relu_of`` (the ReLU's output, same
    shape) the ReLU backward is fused in: ``masked_out = x * (relu_of > 0)``
    is written and ``out`` sums it."""
    if x.dim() != 2:
        raise ValueError("colsum expects a 2-D tensor")
    M, ncol = x.shape
    if out is None:
        out = torch.empty(ncol, dtype=torch.float32, device=x.device)
    if out.dtype != torch.float32 or out.numel() != ncol or not out.is_contiguous():
        raise ValueError("colsum: out must be a contiguous fp32 tensor of x.shape[1] elements")
    if (relu_of is None) != (masked_out is None):
        raise ValueError("colsum: relu_of and masked_out go together")
    if relu_of is not None and (relu_of.shape != x.shape or masked_out.shape != x.shape
                                or masked_out.dtype != x.dtype or not masked_out.is_contiguous()):
        raise ValueError("colsum: relu_of / masked_out must match x (masked_out contiguous)")
    if x.device.type != "cuda" or x.dtype != torch.bfloat16:
        if relu_of is not None:
            torch.where(relu_of > 0, x, torch.zeros_like(x), out=masked_out)
            x = masked_out
        torch.sum(x, 0, dtype=torch.float32, out=out)
        return out
    if M == 0:
        return out.zero_()
    x = x.contiguous()
    if relu_of is not None:
        relu_of = relu_of.contiguous()
    n = _load()
    splits = int(splits or n.colsum_row_splits(M, ncol))
    stream = torch.cuda.current_stream(x.device)
    key = (x.device.index or 0, stream.cuda_stream, ncol, splits)
    ws = _WS.get(key)
    if ws is None:
        # the tickets start at zero and every launch leaves them zero again;
        # one workspace per stream (launches on one stream never overlap)
        ws = (torch.empty((splits, ncol), dtype=torch.float32, device=x.device),
              torch.zeros((ncol + _TILE - 1) // _TILE, dtype=torch.int32, device=x.device))
        _WS[key] = ws
    n.colsum_bf16(out.data_ptr(), x.data_ptr(), M, ncol, ws[0].data_ptr(), ws[1].data_ptr(), splits,
                  stream.cuda_stream, bool(lite), relu_of.data_ptr() if relu_of is not None else 0,
                  masked_out.data_ptr() if masked_out is not None else 0)
    return out
