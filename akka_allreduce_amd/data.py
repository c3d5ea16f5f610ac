"""User I/O contract (reference: ``DataWrapper.scala:3-7``).

``AllReduceInputRequest(iteration)`` -> ``AllReduceInput(data)`` is the data
source; ``AllReduceOutput(data, count, iteration)`` goes to the data sink.

``count`` is the per-element contributor count of the reference
(ReducedDataBuffer.getWithCounts, RB:26-53).  It is carried compactly as one
count per (block, chunk) and expanded to one int32 per element only when the
``count`` attribute is first read (a gfx950 kernel on GPU), so a sink that
never looks at counts does not pay an extra S-element int32 write per round.
"""
from __future__ import annotations

import functools
from dataclasses import dataclass
from typing import Any, Optional

import torch


@dataclass(frozen=True)
class Geometry:
    """Block/chunk layout (W:240-250 with exact integer arithmetic)."""

    dataSize: int
    workerNum: int
    maxChunkSize: int

    @property
    def step(self) -> int:
        return (self.dataSize + self.workerNum - 1) // self.workerNum

    def block_range(self, j: int) -> tuple[int, int]:
        s = min(j * self.step, self.dataSize)
        e = self.dataSize if j >= self.workerNum - 1 else min((j + 1) * self.step, self.dataSize)
        return s, e

    def block_len(self, j: int) -> int:
        s, e = self.block_range(j)
        return e - s

    def num_chunks(self, j: int) -> int:
        return -(-self.block_len(j) // self.maxChunkSize)

    @functools.cached_property
    def kmax(self) -> int:
        return max(1, max(self.num_chunks(j) for j in range(self.workerNum)))

    @functools.cached_property
    def total_chunks(self) -> int:
        return sum(self.num_chunks(j) for j in range(self.workerNum))

    def chunk_range(self, j: int, k: int) -> tuple[int, int]:
        s, e = self.block_range(j)
        cs = s + k * self.maxChunkSize
        return cs, min(cs + self.maxChunkSize, e)

    def expand_counts(self, per_chunk: torch.Tensor) -> torch.Tensor:
        """[N, kmax] counts -> [S] per-element counts (torch reference path)."""
        per_chunk = per_chunk.reshape(self.workerNum, self.kmax)
        idx = torch.arange(self.dataSize, device=per_chunk.device, dtype=torch.int64)
        step = max(self.step, 1)
        blk = torch.clamp(idx // step, max=self.workerNum - 1)
        k = (idx - blk * step) // self.maxChunkSize
        return per_chunk.reshape(-1)[blk * self.kmax + k].to(torch.int32)


@dataclass
class AllReduceInputRequest:
    iteration: int


@dataclass
class AllReduceInput:
    data: Any


class AllReduceOutput:
    """Reduced vector of one round + contributor counts.

    ``data``: 1-D tensor of ``dataSize`` elements (sum over contributors;
    chunks that did not reach the completion threshold are 0).
    ``count``: int32 tensor, per-element contributor count (0 where missing).
    ``iteration``: the round.
    """

    __slots__ = ("data", "iteration", "counts_per_chunk", "geometry", "_count", "_expander", "_event")

    def __init__(
        self,
        data: torch.Tensor,
        count: Optional[torch.Tensor] = None,
        iteration: int = 0,
        *,
        counts_per_chunk: Optional[torch.Tensor] = None,
        geometry: Optional[Geometry] = None,
        expander: Any = None,
        event: Any = None,
    ):
        self.data = data
        self.iteration = iteration
        self.counts_per_chunk = counts_per_chunk
        self.geometry = geometry
        self._count = count
        self._expander = expander
        self._event = event

    @classmethod
    def _make(cls, data: torch.Tensor, iteration: int, counts_per_chunk: torch.Tensor, geometry: "Geometry",
              expander: Any, event: Any) -> "AllReduceOutput":
        """The engine's per-round constructor: positional, no keyword parsing
        (one of these per round; small rounds are priced by their host path)."""
        o = cls.__new__(cls)
        o.data, o.iteration, o.counts_per_chunk, o.geometry = data, iteration, counts_per_chunk, geometry
        o._count, o._expander, o._event = None, expander, event
        return o

    def wait(self) -> "AllReduceOutput":
        """Async rounds: make the current stream wait for the result (no-op otherwise)."""
        if self._event is not None:
            torch.cuda.current_stream(self.data.device).wait_event(self._event)
        return self

    @property
    def count(self) -> torch.Tensor:
        self.wait()
        if self._count is None:
            if self.counts_per_chunk is None or self.geometry is None:
                raise ValueError("AllReduceOutput has no count information")
            if self._expander is not None:
                self._count = self._expander(self.counts_per_chunk)
            else:
                self._count = self.geometry.expand_counts(self.counts_per_chunk)
        return self._count

    def _fused_ok(self, dst: torch.Tensor) -> bool:
        d, g = self.data, self.geometry
        return (d.is_cuda and d.dtype in (torch.float32, torch.bfloat16) and self.counts_per_chunk is not None
                and g is not None and self._count is None and dst.is_contiguous() and dst.dtype == d.dtype
                and dst.device == d.device and dst.numel() == d.numel() and d.data_ptr() % 16 == 0
                and dst.data_ptr() % 16 == 0)

    def _count_mean(self, dst: torch.Tensor, axpy: bool, alpha: float, shadow: Optional[torch.Tensor] = None) -> None:
        from ._native_loader import load

        d, g = self.data, self.geometry
        pc = self.counts_per_chunk.contiguous()
        load().count_mean(dst.data_ptr(), d.data_ptr(), pc.data_ptr(), g.dataSize, g.step, g.workerNum,
                          g.maxChunkSize, g.kmax, "bfloat16" if d.dtype == torch.bfloat16 else "float32",
                          torch.cuda.current_stream(d.device).cuda_stream, axpy, float(alpha),
                          shadow.data_ptr() if shadow is not None else 0)

    def axpy_mean_(self, y: torch.Tensor, alpha: float, shadow: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``y += alpha * mean()`` in one fused pass on the GPU (the SGD update
        of a flat parameter buffer: alpha = -lr); ``y`` is updated in place.
        ``shadow`` (bf16, same length as fp32 ``y``) also receives the updated
        values, stored by the same pass (a separate cast off the fused path)."""
        self.wait()
        if self._fused_ok(y) and (shadow is None or (
                y.dtype == torch.float32 and shadow.dtype == torch.bfloat16 and shadow.is_contiguous()
                and shadow.numel() == y.numel() and shadow.device == y.device and shadow.data_ptr() % 16 == 0)):
            self._count_mean(y, True, alpha, shadow)
            return y
        y.add_(self.mean().view_as(y).to(y.dtype), alpha=alpha)
        if shadow is not None:
            shadow.copy_(y.view_as(shadow))
        return y

    def mean(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Element-wise average over the contributors that made it (0 where none).

        On the GPU this is one fused pass (``count_mean`` kernel: each element
        divided by its chunk's count from the tiny per-chunk table) instead of
        expanding per-element counts; ``out`` may be any same-shape tensor,
        including the buffer that was reduced (gradient buckets)."""
        self.wait()
        d = self.data
        if d.is_cuda:
            dst = torch.empty_like(d) if out is None else out
            if self._fused_ok(dst):
                self._count_mean(dst, False, 0.0)
                return dst
        c = self.count.to(d.dtype if d.is_floating_point() else torch.float32)
        m = torch.where(c > 0, d / c.clamp(min=1), torch.zeros_like(d))
        if out is None:
            return m
        out.copy_(m.view_as(out))
        return out

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"AllReduceOutput(iteration={self.iteration}, n={self.data.numel()}, dtype={self.data.dtype})"
