"""One-sided threshold allreduce: fast ranks never wait for a straggler.

``OneSidedAllreduce`` runs the reference's threshold semantics on the
one-sided lane (csrc/transport/onesided.h, protocol in
csrc/kernels/onesided_protocol.h): every rank exports a window, peers STORE
their scatter chunks and reduced chunks into it, and every send is
fire-and-forget like an Akka ``!`` (AllreduceWorker.scala:227-232, 259-264).

Per call (one round of this rank):

* the round is the rank's next one, unless a peer already pushed a round
  more than ``max_lag`` ahead -- then the call catches up to the oldest round
  still inside the window (W:100-106, implicit start W:164-167);
* each chunk of my block is reduced once floor(thReduce * N) copies landed,
  over exactly the landed set, count = popcount (SB:9-13, SB:20-32);
* the round completes once floor(thComplete * total) reduced chunks landed;
  the others are 0 with count 0 (RB:13-17, RB:26-53, RB:60-66);
* pushes the receiver can no longer use (it already reduced that chunk or
  completed that round) are dropped by the sender (W:155-156, W:172-173).

``out.iteration`` is the round the call served (resolved lazily on the GPU:
reading it waits for the call); ``stats()`` counts drops, forced reduces /
completions, catch-up skips.  GPU ranks (one per MI355X) map each other's
windows through IPC handles; CPU ranks use POSIX shared memory -- the same
protocol code, so multi-process CPU tests cover the GPU's decisions.

Ranks sharing one GPU (tests, rehearsals) that also run compute between
calls should pass ``cu_keep=6``: the round then runs on 6 of every 8 CUs, so
a round waiting on its peers cannot hold every SIMD while a peer's GEMM
needs one (csrc/transport/onesided.h, ``OneSidedParams::cu_keep``).  On a
GPU of its own ``cu_keep=k`` bounds the round's footprint to k of every 8
CUs (its grid sized for them): ``async_op=True`` rounds then overlap compute
on the other CUs (``bounded_footprint``; the DDP hook issues async rounds).
All ``cu_keep`` lanes of a process with the same ``k`` share ONE masked
stream (each extra stream is a hardware queue, csrc/transport/onesided.cpp
``cu_mask_stream``), so their rounds run in issue order: every rank must call
those lanes in the same order (one training loop does), or a rank's later
round queues behind one that waits for a peer still in the other lane.

Usage::

    ar = OneSidedAllreduce(n, max_chunk_size=1 << 20, th_reduce=0.75, th_complete=0.75, max_lag=1)
    out = ar(x)          # AllReduceOutput; out.count / out.mean() as usual
"""
from __future__ import annotations

import os
from typing import Any, Optional

import torch

from .._native_loader import load as _load
from ..utils import tracing as _tracing
from ..data import AllReduceOutput, Geometry
from ..worker import _raw_stream
from .collective import _handle_exchange, env_rank_world

_DTYPES = {torch.float32: "float32", torch.bfloat16: "bfloat16"}
# Hand-off of window bytes between ranks (csrc/kernels/onesided.hip): "lite"
# = write-through stores + drain before each flag, system-coherent loads (no
# cache maintenance); "fenced" = plain stores behind a system-scope release,
# a system-scope acquire after each observed flag -- the HIP memory model's
# own protocol, the fallback for a link on which lite is not proven.
_HANDOFFS = ("lite", "fenced")


class OneSidedOutput(AllReduceOutput):
    """AllReduceOutput whose ``iteration`` (the round served) and ``status``
    come from the lane's per-call record; on the GPU reading them waits for
    the call's kernels (``status_nowait`` reads the record without waiting)."""

    __slots__ = ("_lane", "_call", "_stream", "_status")

    def __init__(self, data, *, lane, call, stream, **kw):
        self._lane = lane
        self._call = call
        self._stream = stream
        self._status = None
        super().__init__(data, **kw)

    @property
    def iteration(self) -> int:  # type: ignore[override]
        return int(self.status["round"])

    @iteration.setter
    def iteration(self, v) -> None:  # the base constructor's placeholder
        pass

    @property
    def call(self) -> int:
        """The lane's id of the call that produced this output."""
        return self._call

    def status_nowait(self) -> dict:
        """The call's record as it is now (host memory the final kernel
        writes): ``round`` is -1 while the call runs.  Raises if the record
        was reused (64 or more later calls)."""
        if self._status is not None:
            return self._status
        if self._call < 0:
            raise RuntimeError("a call captured into a graph has no status record (its replays do)")
        st = self._lane.status(self._call)
        if st["round"] >= 0:
            self._status = st
        return st

    @property
    def status(self) -> dict:
        if self._call < 0:
            raise RuntimeError("a call captured into a graph has no status record (its replays do)")
        if self._status is None:
            if self._stream is not None:  # the raw handle of the stream the call ran on
                dev = self.data.device
                s = torch.cuda.ExternalStream(self._stream, device=dev) if self._stream \
                    else torch.cuda.default_stream(dev)
                s.synchronize()
            st = self._lane.status(self._call)
            if st["round"] < 0:
                raise RuntimeError("onesided call has not finished")
            self._status = st
        return self._status


def _member_exchange(rank: int, members: list, world: int, store: Any, key: str):
    """Like _handle_exchange over ``members`` only: mine -> [bytes of every
    rank], empty for ranks outside the member list."""

    def exchange(mine: bytes) -> list:
        store.set(f"{key}/{rank}", mine)
        return [bytes(store.get(f"{key}/{i}")) if i in members else b"" for i in range(world)]

    return exchange


class OneSidedAllreduce:
    """Threshold allreduce over mapped peer windows (see module docstring)."""

    _instances = 0

    def __init__(
        self,
        data_size: int,
        *,
        max_chunk_size: int = 1 << 20,
        dtype: torch.dtype = torch.float32,
        th_reduce: float = 1.0,
        th_complete: float = 1.0,
        max_lag: int = 1,
        rank: Optional[int] = None,
        world_size: Optional[int] = None,
        device: Optional[torch.device] = None,
        store: Any = None,
        rows: int = 0,
        part_bytes: int = 0,
        timeout_s: float = 30.0,
        threads: int = 256,
        role_wgs: int = 0,
        cu_keep: int = 0,
        data_sink: Any = None,
        handoff: str = "lite",
        members: Optional[list] = None,
        window_output: bool = False,
    ):
        if dtype not in _DTYPES:
            raise ValueError("dtype must be float32 or bfloat16")
        if handoff not in _HANDOFFS:
            raise ValueError(f"handoff must be one of {_HANDOFFS}")
        r, w, local = env_rank_world()
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            r, w = dist.get_rank(), dist.get_world_size()
            local = int(os.environ.get("LOCAL_RANK", str(r)))
        self.rank = r if rank is None else int(rank)
        self.world_size = w if world_size is None else int(world_size)
        if self.world_size < 2:
            raise ValueError("the onesided lane needs N >= 2 ranks")
        if device is None:
            device = torch.device("cuda", local % max(1, torch.cuda.device_count())) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self._cuda = self.device.type == "cuda"
        self._dev_index = (self.device.index if self.device.index is not None else torch.cuda.current_device()) \
            if self._cuda else -1
        self.dtype = dtype
        self.data_size = int(data_size)
        self.geometry = Geometry(self.data_size, self.world_size, int(max_chunk_size))
        self.data_sink = data_sink
        n = _load()
        dev_index = self.device.index if self.device.type == "cuda" else -1
        if dev_index is None:
            dev_index = torch.cuda.current_device()
        self.th_reduce, self.th_complete, self.max_lag = float(th_reduce), float(th_complete), int(max_lag)
        iid = OneSidedAllreduce._instances
        OneSidedAllreduce._instances += 1
        # partial membership (the reference's partial peer map, W:213-216):
        # only ``members`` exchange windows now; the others are never pushed
        # to nor waited for until admit() maps them (re-init, W:87-89)
        self.members = sorted(set(int(q) for q in members) | {self.rank}) if members is not None \
            else list(range(self.world_size))
        partial = len(self.members) < self.world_size
        if partial and store is None:
            raise ValueError("partial membership exchanges windows through a store (late ranks fetch them there)")
        self._store, self._key = store, f"akka/onesided/{iid}"
        exchange = _member_exchange(self.rank, self.members, self.world_size, store, self._key) if partial \
            else _handle_exchange(self.rank, self.world_size, store, self._key)
        # every rank takes part in the exchange even if its own window failed
        # (an empty handle): a local failure raises on EVERY rank, none is
        # left blocked in the collective
        err = None
        try:
            self.lane = n.OneSidedLane(dev_index, self.data_size, self.world_size, int(max_chunk_size), self.rank,
                                       _DTYPES[dtype], th_reduce=float(th_reduce), th_complete=float(th_complete),
                                       max_lag=int(max_lag), rows=int(rows), part_bytes=int(part_bytes),
                                       timeout_ms=int(timeout_s * 1000), threads=int(threads),
                                       role_wgs=int(role_wgs), cu_keep=int(cu_keep),
                                       fenced=handoff == "fenced", window_output=bool(window_output))
            mine = self.lane.handle()
        except Exception as e:  # noqa: BLE001 - re-raised after the exchange
            mine, err = b"", e
        handles = exchange(mine)
        if err is not None:
            raise err
        missing = [i for i, h in enumerate(handles) if not h and i in self.members]
        if missing:
            raise RuntimeError(f"onesided lane: ranks {missing} could not create their windows")
        self.lane.open(handles)
        if members is not None and store is not None:
            # a membership that may grow (admit): ranks joining later open
            # this window by name / handle, so it stays published (CPU: the
            # shm name is removed when the lane goes)
            _member_exchange(self.rank, self.members, self.world_size, store, f"{self._key}/opened")(b"1")
        else:
            # every rank mapped every window: names may go (a killed rank leaves no shm behind)
            exchange_done = _handle_exchange(self.rank, self.world_size, store, f"{self._key}/opened")
            exchange_done(b"1")
            self.lane.unlink()
        self._kmax = self.geometry.kmax
        # counts tables reused with caller-owned outputs, one per output buffer
        # (a caller alternating buffers keeps each round's counts with its data)
        self._counts: dict = {}
        self._side: Optional[torch.cuda.Stream] = None  # async_op rounds
        self.calls = 0
        # window output (exact rounds): a call without ``out`` returns the
        # gather row of its call id in this rank's own window -- the peers'
        # reduced parts land there in place, no copy -- valid until the NEXT
        # call of this lane (like a reused ``out``)
        self._rows: Optional[list] = None
        if self.lane.info().get("window_output"):
            from torch.utils.dlpack import from_dlpack

            dname = _DTYPES[dtype]
            self._rows = [from_dlpack(self.lane.gather_row_dlpack(d, dname, int(dev_index)))
                          for d in range(int(self.lane.info()["rows"]))]

    def __call__(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, async_op: bool = False) -> OneSidedOutput:
        """One round of this rank.  GPU: enqueued on the current stream (the
        output is valid in its order).  ``async_op=True`` (GPU): the round runs
        on the lane's side stream, behind everything enqueued so far on the
        current one, so later work on the current stream (the rest of a
        backward pass) overlaps it; ``wait()`` -- or ``mean()`` / ``count`` /
        ``axpy_mean_()``, which call it -- joins the result into the then
        current stream (torch.distributed's ``async_op`` convention).
        CPU: returns after the round completed."""
        if x.numel() != self.data_size:
            raise ValueError(f"expected {self.data_size} elements, got {x.numel()}")
        if x.dtype != self.dtype or x.device != self.device:
            x = x.to(device=self.device, dtype=self.dtype)
        if x.dim() != 1 or not x.is_contiguous():
            x = x.reshape(-1).contiguous()
        reuse = out is not None
        lane_out = out is None and self._rows is not None and self.data_sink is None
        if lane_out:
            # refused BEFORE the launch: a round enqueued into the capture
            # would replay with no Python output and shift the call ids
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("a captured call needs an output buffer (out=...)")
            out = None  # the kernel writes the window row of this call's id
        elif out is None:
            out = torch.empty_like(x)
        elif out.numel() != self.data_size or out.dtype != self.dtype or not out.is_contiguous():
            raise ValueError("out must be a contiguous tensor of the buffer's size and dtype")
        if reuse:
            # the caller manages the output's lifetime (``out`` given): the
            # counts table is reused with THAT buffer, like the buffer itself
            key = out.data_ptr()
            counts = self._counts.get(key)
            if counts is None:
                if len(self._counts) >= 16:  # bounded: buffers a caller dropped
                    self._counts.pop(next(iter(self._counts)))
                counts = torch.empty((self.world_size, self._kmax), dtype=torch.int32, device=self.device)
                self._counts[key] = counts
        else:
            counts = torch.empty((self.world_size, self._kmax), dtype=torch.int32, device=self.device)
        # (a raw stream handle: building a Stream object per call costs ~1.7 us,
        # profiles/r06/small_rounds/)
        stream = _raw_stream(self._dev_index) if self._cuda else None
        event = None
        if async_op and stream is not None:
            side = self._side_stream()
            side.wait_stream(torch.cuda.current_stream(self.device))
            for t in (x, counts) + ((out,) if out is not None else ()):  # in use on the side stream too
                t.record_stream(side)
            stream = side.cuda_stream
        # roctx range around the enqueue (AKKA_TRACE=1; rocprofv3 --marker-trace)
        if _tracing._enabled:
            with _tracing.range_(f"akka.onesided call {self.calls}"):
                call = self.lane.round(stream if stream is not None else 0, x.data_ptr(),
                                       0 if lane_out else out.data_ptr(), counts.data_ptr(), self._kmax)
        else:
            call = self.lane.round(stream if stream is not None else 0, x.data_ptr(),
                                   0 if lane_out else out.data_ptr(), counts.data_ptr(), self._kmax)
        if lane_out:
            if call < 0:
                raise RuntimeError("a captured call needs an output buffer (out=...)")
            out = self._rows[call % len(self._rows)][: self.data_size]
        if async_op and stream is not None:
            event = torch.cuda.Event()
            event.record(self._side)
        if call >= 0:  # (a captured call counts once per replay: note_replays)
            self.calls += 1
        o = OneSidedOutput(out.view(-1), lane=self.lane, call=call, stream=stream, counts_per_chunk=counts,
                           geometry=self.geometry, expander=self._expand if stream is not None else None,
                           event=event)
        if self.data_sink is not None:
            self.data_sink(o)
        return o

    def _side_stream(self) -> "torch.cuda.Stream":
        if self._side is None:
            if self.bounded_footprint:
                # the lane's CU-masked stream itself (shared by the process's
                # lanes): async rounds launch there with no fork / join
                self._side = torch.cuda.ExternalStream(int(self.lane.cu_stream()), device=self.device)
            else:
                self._side = torch.cuda.Stream(self.device)
        return self._side

    @property
    def capturable(self) -> bool:
        """A call can be captured in a HIP graph (GPU): its launches take the
        same arguments every call (with ``out`` given) and the lane's round /
        call sequence lives in device memory.  After each replay of a captured
        call, ``note_replays(1)`` keeps the host's call ids in step."""
        return self.device.type == "cuda" and self.data_sink is None

    @property
    def window_output(self) -> bool:
        """Calls without ``out`` return a window row (valid until the next call)."""
        return self._rows is not None

    @property
    def bounded_footprint(self) -> bool:
        """The round runs on a subset of the CUs of a GPU of its own
        (``cu_keep``): an async round leaves the other CUs to the kernels it
        overlaps (the DDP backward), so a hook should issue async rounds."""
        b = getattr(self, "_bounded", None)
        if b is None:  # fixed once the windows are open
            i = self.lane.info()
            dedicated = int(i.get("ranks_on_this_gpu", 1)) <= 1 or os.environ.get("AKKA_OS_DEDICATED") == "1"
            b = self._bounded = int(i.get("lane_cus", 0)) > 0 and dedicated
        return b

    @property
    def handoff(self) -> str:
        return "fenced" if self.lane.fenced else "lite"

    def set_handoff(self, mode: str) -> None:
        """Hand-off mode of this rank's later calls ("lite" / "fenced"); the
        modes share the protocol's tags, so ranks may switch independently."""
        if mode not in _HANDOFFS:
            raise ValueError(f"handoff must be one of {_HANDOFFS}")
        self.lane.set_fenced(mode == "fenced")

    def admit(self, peer: int, timeout_s: float = 60.0) -> None:
        """Re-init with a larger peer map (W:87-89): map ``peer``'s window
        (published in the store when it created its lane) and push to / wait
        for it from the next call on.  Between calls only (synchronises the
        device).  A rank already mapped raises."""
        import time

        q = int(peer)
        if q in self.members:
            return
        if self._store is None:
            raise ValueError("admit: windows of late ranks come through the store given at construction")
        t0 = time.monotonic()
        while True:  # the joining rank may still be creating its window
            try:
                h = bytes(self._store.get(f"{self._key}/{q}"))
                break
            except Exception:  # noqa: BLE001 - store timeout: retry until ours expires
                if time.monotonic() - t0 > timeout_s:
                    raise
        if not h:
            raise RuntimeError(f"onesided lane: rank {q} could not create its window")
        self.lane.add_peer(q, h)
        self.members = sorted(self.members + [q])

    def note_replays(self, n: int) -> None:
        self.lane.note_replays(int(n))
        self.calls += int(n)

    def _expand(self, per_chunk: torch.Tensor) -> torch.Tensor:
        g = self.geometry
        out = torch.empty(g.dataSize, dtype=torch.int32, device=per_chunk.device)
        _load().count_expand(out.data_ptr(), per_chunk.contiguous().data_ptr(), g.dataSize, g.step, g.workerNum,
                             g.maxChunkSize, g.kmax, torch.cuda.current_stream(per_chunk.device).cuda_stream)
        return out

    # ---- control / observability ------------------------------------------------
    def stats(self) -> dict:
        """Lane counters (GPU: synchronises the device)."""
        return dict(self.lane.stats())

    def info(self) -> dict:
        return dict(self.lane.info())

    def error(self) -> int:
        """Non-zero once a bounded wait expired (that round was forced; its
        counts are still honest)."""
        return int(self.lane.error())

    def mark_dead(self, peer: int, dead: bool = True) -> None:
        """Never wait for (nor write to) ``peer`` again -- e.g. on the master's
        WorkerTerminated (M:46-52)."""
        self.lane.set_dead(int(peer), bool(dead))

    def force_below(self, round_plus_one: int) -> None:
        """Force every round < ``round_plus_one`` (waits end with what landed)."""
        self.lane.force_below(int(round_plus_one))

    def retire(self) -> None:
        """This rank serves no further round: peers stop waiting for its
        copies of later rounds (the job's end, like the master's maxRound)."""
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
        self.lane.retire(stream)

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
