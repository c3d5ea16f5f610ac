"""torch DDP communication hook: gradient buckets through the threshold allreduce.

    from akka_allreduce_amd.parallel.ddp import ThresholdHookState, threshold_allreduce_hook
    model = DistributedDataParallel(model, gradient_as_bucket_view=True)
    model.register_comm_hook(ThresholdHookState(th_reduce=0.75, th_complete=0.75), threshold_allreduce_hook)

(``gradient_as_bucket_view=True``: the hook writes the mean into the bucket
in place, so the gradients -- views of the buckets -- need no copy back.)

Every DDP bucket becomes one round of a ``ThresholdAllreduce`` (one per
distinct bucket size, created lazily -- all ranks see the same bucket sequence,
so creation is collective-safe).  The bucket is replaced by the mean over the
contributors that made it into the round (per-element ``count``), which is
what DDP's default hook computes at thresholds 1 (sum / world size) and stays
unbiased when a straggler's gradients are missing (``count`` lets
a consumer average partial sums).  With ``transport="onesided"`` the fast
ranks never wait for a live straggler (device-side thresholds over mapped
windows, parallel/onesided.py; one window set per bucket size, since each
lane's round tags are its own); ``transport="reactive"`` is the RCCL
alternative, bounded by its send-slot pool.
"""
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .collective import ThresholdAllreduce


class ThresholdHookState:
    """``async_op`` (default True): on GPUs the hook returns before the round
    ran -- the round, the count-weighted mean and the future's ready event are
    all queued in stream order (DDP waits on the future's CUDA event, not on
    the host), so bucket communication overlaps the rest of the backward pass
    like DDP's own allreduce hook.  ``th_allreduce``: master-style round
    pacing across ranks (see ThresholdAllreduce).  ``data_plane="ipc"``: exact
    rounds on the one-sided xGMI lane, no RCCL communicator (ThresholdAllreduce).
    ``tune`` (exact thresholds): the hook's first engine measures every exact
    lane once and keeps the fastest; later engines take the same lane
    (ThresholdAllreduce.tune).

    One transport per hook (scheduled ``stream`` transport): the engines of
    the different bucket sizes share the first engine's device streams and
    communicator
    (``share_transport_with``), so a job holds ONE RCCL communicator however
    many bucket shapes DDP produces, and every bucket's round is ordered on the
    same streams in the bucket order every rank sees.  With the ipc data plane
    the engines also share the first engine's window memory when it is large
    enough (``ipc_capacity``: the window is sized for ``bucket_cap_mb``).
    Reactive engines keep one transport each (their phase-2 groups are issued
    in a timing-dependent order, which two engines must not interleave on one
    pair communicator)."""

    def __init__(self, *, th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 2,
                 max_chunk_size: int = 1 << 20, transport: str = "stream", broadcast_lag: int = 2,
                 async_op: bool = True, th_allreduce=None, data_plane: str = "rccl", tune: bool = False,
                 bucket_cap_mb: float = 25.0, onesided_options: Optional[dict] = None):
        self.kw = dict(th_reduce=th_reduce, th_complete=th_complete, max_lag=max_lag, max_chunk_size=max_chunk_size,
                       transport=transport, broadcast_lag=broadcast_lag, th_allreduce=th_allreduce,
                       data_plane=data_plane, onesided_options=onesided_options)
        self.engines: Dict[Tuple[int, torch.dtype, torch.device], ThresholdAllreduce] = {}
        self.rounds = 0
        self.async_op = async_op
        self.async_rounds = 0
        self.tune = tune and th_reduce >= 1.0 and th_complete >= 1.0
        self.bucket_cap_bytes = int(bucket_cap_mb * (1 << 20))
        self.first: Dict[Tuple[torch.dtype, torch.device], ThresholdAllreduce] = {}
        self.lane = None  # tuned lane, applied to every engine

    def engine(self, t: torch.Tensor) -> ThresholdAllreduce:
        key = (t.numel(), t.dtype, t.device)
        ar = self.engines.get(key)
        if ar is None:
            first = self.first.get((t.dtype, t.device))
            cap = max(t.numel(), self.bucket_cap_bytes // t.element_size())
            # one transport per hook only for the scheduled link: reactive
            # engines drive their pair communicators from per-peer streams in
            # a timing-dependent order, so each keeps its own
            share = first if self.kw["transport"] == "stream" else None
            ar = ThresholdAllreduce(t.numel(), dtype=t.dtype, device=t.device, share_transport_with=share,
                                    ipc_capacity=cap, **self.kw)
            if first is None:
                self.first[(t.dtype, t.device)] = ar
            if ar.world_size > 1 and ar.transport == "stream":
                if self.tune and self.lane is None:
                    self.lane = ar.tune()["chosen"]  # collective: every rank creates this engine at the same bucket
                elif self.lane is not None:  # tuned once per hook: later engines take the same lane
                    if self.lane.startswith("ipc") and not ar.state().get("link", {}).get("ipc"):
                        ar.enable_ipc()  # collective, like the engine's creation
                    ar.use_lane(self.lane)
            self.engines[key] = ar
        return ar

    def transports(self) -> int:
        """Distinct transports (communicators) the hook's engines use."""
        return len({ar.worker._core.transport_id() for ar in self.engines.values() if ar.worker is not None})


# (real annotations, not postponed strings: DDP checks them)
def threshold_allreduce_hook(state: ThresholdHookState, bucket: dist.GradBucket) -> torch.futures.Future[torch.Tensor]:
    t = bucket.buffer()
    flat = t.reshape(-1)
    if flat.dtype not in (torch.float32, torch.bfloat16):
        work = flat.float()
    else:
        work = flat
    ar = state.engine(work)
    cuda = work.is_cuda
    async_op = bool(state.async_op and cuda and ar.runs_async())
    out = ar(work.contiguous(), async_op=async_op)
    state.rounds += 1
    state.async_rounds += int(async_op)
    if not cuda:
        fut: torch.futures.Future[torch.Tensor] = torch.futures.Future()
        fut.set_result(out.mean().to(t.dtype).view_as(t))
        return fut
    # CUDA-aware future: set_result records an event on the stream current at
    # that point, and DDP's wait() makes ITS stream wait on that event (and
    # record_streams the result).  Async: the count-mean runs on the engine's
    # compute stream behind the round, so the caller's stream -- the rest of
    # the backward pass -- only waits where DDP consumes the bucket.
    side = ar.async_stream() if async_op else torch.cuda.current_stream(work.device)
    with torch.cuda.stream(side):
        if work is flat and t.is_contiguous() and ar.transport != "reactive":
            # the mean straight into the bucket (the round is done with its
            # input by then, in this stream's order): no allocation, and the
            # result aliases the bucket, so DDP's copy of it into the
            # gradients is a no-op with gradient_as_bucket_view=True.  (Not
            # reactive: its round may complete while a send of the input to
            # a straggler is still in flight.)
            mean = out.mean(out=flat).view_as(t)
        else:
            mean = out.mean().to(t.dtype).view_as(t)
        fut = torch.futures.Future(devices=[work.device])
        fut.set_result(mean)
    return fut
