"""Python entry points for the chunk N-way sum and the count expansion.

``chunk_reduce`` is hot spot K1 of SURVEY §2.3 (reference:
ScatteredDataBuffer.reduce, SB:20-32) as a standalone op.  CUDA tensors always
go to the native gfx950 kernel (there is no silent fallback: a missing
extension raises); CPU tensors use a plain torch sum, which is also the
numerics reference the GPU tests compare against.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .._native_loader import load as _load
from ..data import Geometry

_DT = {torch.float32: "float32", torch.bfloat16: "bfloat16"}


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def chunk_reduce(srcs: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None, impl: str = "auto") -> torch.Tensor:
    """``out = sum(srcs)`` elementwise, fp32 accumulation, output in the inputs' dtype.

    ``impl``: ``auto`` | ``vec`` (16-B loads to VGPRs, cache policy picked from
    the working set) | ``vec_nts`` / ``vec_ntl`` / ``vec_both`` (vec with a fixed
    nontemporal-store / -load / both policy) | ``lds`` (LDS-DMA staged)
    | ``scalar``.  All sources must share shape, dtype and device.
    """
    if len(srcs) == 0:
        raise ValueError("chunk_reduce needs at least one source")
    ref = srcs[0]
    for s in srcs:
        if s.shape != ref.shape or s.dtype != ref.dtype or s.device != ref.device:
            raise ValueError("chunk_reduce sources must share shape, dtype and device")
    if ref.dtype not in _DT:
        raise TypeError(f"unsupported dtype {ref.dtype}")
    if out is None:
        out = torch.empty_like(ref)
    if ref.device.type != "cuda":
        acc = torch.zeros(ref.shape, dtype=torch.float32)
        for s in srcs:
            acc += s.float()
        out.copy_(acc.to(ref.dtype))
        return out
    n = _load()
    srcs = [s.contiguous() for s in srcs]
    if not out.is_contiguous():
        raise ValueError("out must be contiguous")
    n.reduce(out.data_ptr(), [s.data_ptr() for s in srcs], ref.numel(), _DT[ref.dtype], _stream(ref), impl)
    return out


def count_expand(per_chunk: torch.Tensor, geometry: Geometry) -> torch.Tensor:
    """[N, kmax] per-chunk contributor counts -> [S] per-element counts (RB:41-47)."""
    per_chunk = per_chunk.to(torch.int32).contiguous()
    if per_chunk.numel() != geometry.workerNum * geometry.kmax:
        raise ValueError("per_chunk must have workerNum * kmax entries")
    if per_chunk.device.type != "cuda":
        return geometry.expand_counts(per_chunk)
    n = _load()
    out = torch.empty(geometry.dataSize, dtype=torch.int32, device=per_chunk.device)
    n.count_expand(out.data_ptr(), per_chunk.data_ptr(), geometry.dataSize, geometry.step, geometry.workerNum,
                   geometry.maxChunkSize, geometry.kmax, _stream(per_chunk))
    return out
