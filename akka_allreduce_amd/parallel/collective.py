"""SPMD front end: one process per GPU (torchrun), RCCL p2p over xGMI.

``ThresholdAllreduce`` wraps one ``AllreduceWorker`` per rank on the scheduled
(``stream``) transport.  Every rank starts round r when it calls the object
(each rank is its own master for pacing; with ``thAllreduce = 1`` and
lock-step callers this is exactly the reference's master behaviour, M:54-63,
without a control-plane round trip per round -- or, with ``th_allreduce``,
paced through the store like the reference's master).  The RCCL unique id is shared
through ``torch.distributed`` (any backend; gloo is enough) or a TCPStore.

Usage::

    ar = ThresholdAllreduce(data_size=x.numel(), max_chunk_size=1 << 20)
    out = ar(x)          # AllReduceOutput; out.data is valid in stream order

``lane`` picks how exact-threshold rounds (thReduce = thComplete = 1) move:
``"auto"`` / ``"p2p"`` run the chunk-pipelined p2p schedule with the gfx950
reduce, ``"ipc"`` the one-sided kernels over mapped peer windows (after
``enable_ipc``), ``"collective"`` RCCL's own reduce-scatter + all-gather -- a
comparator only, never chosen automatically (``tune`` picks among the
framework's lanes).  Rounds with thresholds < 1 always take the p2p schedule
(their outcome depends on arrival order).

``th_allreduce`` adds the reference's third straggler knob, the master's
round pacing (M:54-63): a rank starts round r only once ``thAllreduce * N``
ranks completed round r-1 (counters in the job's TCPStore, no master
process); on the onesided transport a call also reports the rounds it skipped
by catch-up as completed.  ``None`` (default): each rank paces itself.

``transport="onesided"`` is the straggler-tolerant path of choice
(parallel/onesided.py, csrc/transport/onesided.h): every send is a store into
the receiver's mapped window, so no rank ever waits for a slow one, in steady
state.  ``transport="reactive"`` is the two-sided alternative
(csrc/transport/reactive_link.h): one stream + one RCCL pair communicator per
peer, arrivals polled from events; a lagging peer pins one send slot per
round, so after the slot pool (16) the fast ranks run at its pace.  It runs
N+2 streams per process: set ``GPU_MAX_HW_QUEUES`` (<= 32) to at least N+4
before the first HIP call, or parked streams share hardware queues.
"""
from __future__ import annotations

import os
import time
from typing import Any, Optional

import torch

from .._native_loader import load as _load
from ..data import AllReduceOutput
from ..messages import InitWorkers
from ..worker import AllreduceWorker, _raw_stream


class _RemoteRank:
    """Placeholder reference for a peer rank: the scheduled transport never tells it anything."""

    def __init__(self, rank: int):
        self.rank = rank

    def tell(self, msg: Any, sender: Any = None) -> None:  # pragma: no cover - never called
        raise RuntimeError(f"message {type(msg).__name__} routed to remote rank {self.rank} outside RCCL")


def env_rank_world() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def share_unique_id(rank: int, world: int, store: Any = None) -> bytes:
    """RCCL unique id from rank 0 to everyone (torch.distributed or a TCPStore)."""
    n = _load()
    if world == 1:
        return b""
    if store is not None:
        if rank == 0:
            store.set("akka/rccl_uid", n.rccl_unique_id())
        return bytes(store.get("akka/rccl_uid"))
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("initialise torch.distributed (gloo is enough) or pass a TCPStore to share the RCCL id")
    obj = [n.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def _handle_exchange(rank: int, world: int, store: Any, key: str):
    """A function mine -> [every rank's bytes] over the store or torch.distributed."""

    def exchange(mine: bytes) -> list:
        if store is not None:
            store.set(f"{key}/{rank}", mine)
            return [bytes(store.get(f"{key}/{i}")) for i in range(world)]
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("exchanging window handles needs torch.distributed (gloo is enough) or a store")
        out = [None] * world
        dist.all_gather_object(out, mine)
        return out

    return exchange


class RoundPacer:
    """The master's round pacing (M:54-63) without a master process: round r
    may start on a rank once at least ``thAllreduce * N`` ranks (float32
    product, like the reference) completed round r-1.  Completions are
    counters in the job's key-value store (torch.distributed's TCPStore,
    hosted by rank 0), so pacing costs one store add per round plus polls
    while a rank is ahead of the threshold."""

    def __init__(self, store: Any, prefix: str, world: int, th_allreduce: float, timeout: float = 300.0):
        import numpy as np

        self.store = store
        self.prefix = prefix
        self.world = int(world)
        self.need = float(np.float32(world) * np.float32(th_allreduce))
        self.timeout = timeout
        self.waited_s = 0.0
        self.waits = 0

    def completed(self, r: int) -> None:
        self.store.add(f"{self.prefix}/{r}", 1)

    def wait_start(self, r: int, progress: Any = None) -> None:
        """Block until round ``r`` may start (always for r = 0).  ``progress``
        (e.g. the reactive worker's poll) keeps this rank's own transfers
        moving while it waits: the ranks being waited for may need them."""
        if r <= 0:
            return
        import time

        key = f"{self.prefix}/{r - 1}"
        t0 = time.monotonic()
        nap = 2e-5
        while self.store.add(key, 0) < self.need:
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"round {r}: fewer than {self.need:g} ranks completed round {r - 1} "
                                   f"within {self.timeout:g} s (thAllreduce pacing)")
            if progress is not None and progress():
                nap = 2e-5
                continue
            time.sleep(nap)
            nap = min(nap * 2, 2e-3)
        dt = time.monotonic() - t0
        if dt > 1e-4:
            self.waits += 1
        self.waited_s += dt
        # Key r-1 is read only by ranks starting round r.  The last of the N
        # ranks to pass here removes it (and its own pass counter), so the
        # store hosted by rank 0 does not grow by a key per round forever.
        passed = f"{self.prefix}/passed/{r - 1}"
        if self.store.add(passed, 1) >= self.world:
            for k in (key, passed):
                try:
                    self.store.delete_key(k)
                except Exception:  # noqa: BLE001 - a store without deletion keeps the keys
                    pass


class ThresholdAllreduce:
    _instances = 0  # creation order is the same on every rank: names pacing keys

    def __init__(
        self,
        data_size: int,
        *,
        max_chunk_size: int = 1 << 20,
        dtype: torch.dtype = torch.float32,
        th_reduce: float = 1.0,
        th_complete: float = 1.0,
        max_lag: int = 2,
        broadcast_lag: int = 2,
        rank: Optional[int] = None,
        world_size: Optional[int] = None,
        device: Optional[torch.device] = None,
        store: Any = None,
        data_sink: Any = None,
        transport: str = "stream",
        lane: str = "auto",
        th_allreduce: Optional[float] = None,
        data_plane: str = "rccl",
        share_transport_with: Optional["ThresholdAllreduce"] = None,
        ipc_capacity: int = 0,
        onesided_options: Optional[dict] = None,
    ):
        # extra OneSidedAllreduce arguments for the one-sided lane (transport
        # "onesided" or lane "onesided"), e.g. {"cu_keep": 6} on a shared GPU
        self.onesided_options = dict(onesided_options or {})
        self._lane_os = False  # exact rounds on the one-sided lane (use_lane("onesided"))
        self._ipc_direct = False  # exact ipc rounds straight on the caller's stream (use_lane("*_direct"))
        self._ipc_dev_on = False  # the ipc lane's round id lives on the device
        self._direct = None    # an open CapturableExact view
        # direct ipc rounds: the last workgroup writes the counts table (like
        # an engine round) instead of zeroing it on failure only (measurement
        # knob of bench/small_rounds.py, AKKA_IPC_DIRECT_FINISH=1)
        self._ipc_finish = os.environ.get("AKKA_IPC_DIRECT_FINISH") == "1"
        if transport == "onesided":
            # thresholds over mapped peer windows: no send ever waits for a
            # peer (parallel/onesided.py, csrc/transport/onesided.h)
            from ..utils.faults import env_straggler_delay
            from .onesided import OneSidedAllreduce

            self._os = OneSidedAllreduce(data_size, max_chunk_size=max_chunk_size, dtype=dtype, th_reduce=th_reduce,
                                         th_complete=th_complete, max_lag=max_lag, rank=rank, world_size=world_size,
                                         device=device, store=store, data_sink=data_sink, **self.onesided_options)
            self.rank, self.world_size, self.device = self._os.rank, self._os.world_size, self._os.device
            self.transport, self.worker, self.pacer, self.store = "onesided", None, None, store
            self.data_size, self._round = int(data_size), 0
            self.fault_delay_s = env_straggler_delay(self.rank)
            self._max_lag = int(max_lag)
            if th_allreduce is not None and self.world_size > 1:
                # the master's pacing (M:54-63) on top of the lane's catch-up:
                # round r starts once thAllreduce * N ranks completed r - 1
                pstore = store
                if pstore is None:
                    import torch.distributed as dist

                    if not dist.is_initialized():
                        raise RuntimeError("thAllreduce pacing needs torch.distributed initialised or a store")
                    pstore = dist.distributed_c10d._get_default_store()
                ThresholdAllreduce._instances += 1
                self.pacer = RoundPacer(pstore, f"akka/pace/os/{ThresholdAllreduce._instances}", self.world_size,
                                        float(th_allreduce))
            return
        if transport not in ("stream", "reactive"):
            raise ValueError("transport must be 'stream', 'reactive' or 'onesided'")
        if data_plane not in ("rccl", "ipc", "ipc_p2p"):
            raise ValueError("data_plane must be 'rccl', 'ipc' or 'ipc_p2p'")
        if data_plane == "ipc" and (transport != "stream" or th_reduce < 1.0 or th_complete < 1.0):
            raise ValueError("the ipc-only data plane runs exact rounds (thresholds 1) on the stream transport")
        r, w, local = env_rank_world()
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            # an initialised process group is authoritative (mp.spawn sets no RANK/WORLD_SIZE env)
            r, w = dist.get_rank(), dist.get_world_size()
            local = int(os.environ.get("LOCAL_RANK", str(r)))
        self.rank = r if rank is None else int(rank)
        self.world_size = w if world_size is None else int(world_size)
        if device is None:
            device = torch.device("cuda", local % max(1, torch.cuda.device_count())) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        if data_plane != "rccl" and self.device.type != "cuda":
            raise ValueError("the ipc-only data plane maps peer GPU memory: it needs a cuda device")
        if transport == "reactive" and self.world_size > 1 and self.device.type == "cuda":
            need = min(32, self.world_size + 4)
            have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
            if have < need:
                raise RuntimeError(f"reactive transport at N={self.world_size} needs GPU_MAX_HW_QUEUES >= {need} "
                                   f"(have {have}); export it (<= 32) before the first HIP call")
        share = share_transport_with if self.world_size > 1 else None
        if share is not None:
            # ride on another engine's transport: one communicator (and one set
            # of device streams) for every engine of the job, e.g. one per DDP
            # bucket size (WorkerCore.adopt_transport)
            if transport != "stream":
                raise ValueError("share_transport_with: only the scheduled (stream) transport can be shared "
                                 "(reactive links issue groups in a timing-dependent order)")
            if (share.transport != transport or share.device != self.device or share.world_size != self.world_size
                    or share.rank != self.rank or getattr(share, "data_plane", data_plane) != data_plane):
                raise ValueError("share_transport_with: the engines differ in transport, device, rank or data plane")
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device)
            spec = ("shared", share.worker)
        elif self.device.type == "cuda" and data_plane == "ipc" and self.world_size > 1:
            torch.cuda.set_device(self.device)
            spec = ("none", self.rank, self.world_size)
        elif self.device.type == "cuda" and data_plane == "ipc_p2p" and self.world_size > 1:
            # every schedule (thresholds, reactive) over mailboxes in mapped peer
            # memory instead of RCCL (csrc/transport/ipc_p2p.cpp)
            torch.cuda.set_device(self.device)
            spec = ("ipc_p2p", self.rank, self.world_size,
                    _handle_exchange(self.rank, self.world_size, store, f"akka/p2p/{ThresholdAllreduce._instances}"))
        elif self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            uid = share_unique_id(self.rank, self.world_size, store)
            spec = ("rccl", uid, self.rank, self.world_size) if self.world_size > 1 else ("local",)
        else:
            # CPU processes: the same schedules over torch.distributed (gloo) p2p
            from .gloo import make_async_fns, make_group_fn

            if self.world_size == 1:
                spec = ("local",)
            elif transport == "reactive":
                # one gloo group per reactive engine: its pair transfers can
                # outlive a call and gloo matches by (peer, tag), so another
                # engine's transfers must never share the group (like one
                # RCCL pair communicator set per engine on the GPU)
                grp = dist.new_group(backend="gloo") if dist.is_initialized() else None
                post, test = make_async_fns(grp)
                spec = ("async_callback", post, test, self.rank, self.world_size)
            else:
                spec = ("callback", make_group_fn(), self.rank, self.world_size)
        self.transport = transport if self.world_size > 1 else "stream"
        self.worker = AllreduceWorker(None, data_sink, device=self.device, dtype=dtype, transport=self.transport,
                                      transport_spec=spec, broadcast_lag=broadcast_lag, strict=True,
                                      name=f"rank{self.rank}")
        peers = {i: (self.worker if i == self.rank else _RemoteRank(i)) for i in range(self.world_size)}
        self.worker.tell(InitWorkers(peers, self.world_size, None, self.rank, th_reduce, th_complete, max_lag,
                                     int(data_size), int(max_chunk_size)))
        self.data_size = int(data_size)
        self.store = store
        self.data_plane = data_plane
        self._share = share
        self._ipc_capacity = int(ipc_capacity)
        self._iid = ThresholdAllreduce._instances
        self._ipc_epoch = 0
        self._exact_os = None  # the one-sided lane at thresholds 1 (lane "onesided")
        self._th_exact = th_reduce >= 1.0 and th_complete >= 1.0
        if data_plane == "ipc" and self.world_size > 1:
            self.enable_ipc()
            lane = "ipc"
        if self.transport == "stream":
            self.worker.set_lane(lane)
        from ..utils.faults import env_straggler_delay

        self.fault_delay_s = env_straggler_delay(self.rank)  # AKKA_FAULT_RANK / AKKA_FAULT_DELAY_MS
        ThresholdAllreduce._instances += 1
        self.pacer: Optional[RoundPacer] = None
        if th_allreduce is not None and self.world_size > 1:
            pstore = store
            if pstore is None:
                import torch.distributed as dist

                if not dist.is_initialized():
                    raise RuntimeError("thAllreduce pacing needs torch.distributed initialised or a store")
                pstore = dist.distributed_c10d._get_default_store()
            self.pacer = RoundPacer(pstore, f"akka/pace/{ThresholdAllreduce._instances}", self.world_size,
                                    float(th_allreduce))
        self._round = 0

    def __call__(self, x: torch.Tensor, async_op: bool = False, out: Optional[torch.Tensor] = None) -> AllReduceOutput:
        """One round.  ``async_op=True``: call ``.wait()`` before reading ``.data``.
        ``out``: preallocated output buffer (reused across rounds)."""
        if x.numel() != self.data_size:
            raise ValueError(f"expected {self.data_size} elements, got {x.numel()}")
        w = self.worker
        if (w is not None and self.pacer is None and self._direct is None and not self._lane_os
                and not self._ipc_direct and not self.fault_delay_s and w._fast_ok(x)):
            # the common call: straight into the worker's native fast path
            # (small rounds are priced by this host path, profiles/r06/small_rounds/)
            o = w._fast_allreduce(x, async_op, out)
            if o is None:
                raise RuntimeError("round did not complete (thresholds need every rank in the scheduled transport)")
            self._round += 1
            return o
        if self.fault_delay_s:
            import time

            time.sleep(self.fault_delay_s)
        r = self._round
        if self.transport == "onesided":
            if self.pacer is None:
                self._round += 1
                # (async_op: the round is valid in the caller's stream order,
                # which satisfies wait(); a side stream only adds hand-offs --
                # unless the round's footprint is bounded, see runs_async)
                return self._os(x, out=out, async_op=async_op and self._os.bounded_footprint)
            # paced: wait for round r, call, then report every round this call
            # completed -- the served one and any it skipped by catch-up (the
            # reference force-completes those, W:100-106) -- like
            # CompleteAllreduce to the master (W:276)
            self.pacer.wait_start(r)
            o = self._os(x, out=out)
            served = o.iteration  # waits for the call
            for rr in range(r, served + 1):
                self.pacer.completed(rr)
            self._round = served + 1
            return o
        if self.pacer is not None:
            self.pacer.wait_start(r, self.worker.poll if self.transport == "reactive" else None)
        if self._direct is not None:
            raise RuntimeError("this engine's rounds run through its capturable view now (close() it first)")
        if self._lane_os:
            # exact rounds on the one-sided lane (tune candidate "onesided"):
            # valid in the caller's stream order, like an async round
            out = self._exact_os(x, out=out, async_op=async_op and self._exact_os.bounded_footprint)  # (see above)
        elif getattr(self, "_ipc_direct", False):
            out = self._ipc_direct_round(x, out)  # valid in the caller's stream order (satisfies wait())
        else:
            out = self.worker.allreduce(x, async_op=async_op, out=out)
        if out is None:
            raise RuntimeError("round did not complete (thresholds need every rank in the scheduled transport)")
        self._round += 1
        if self.pacer is not None:
            self.pacer.completed(r)  # CompleteAllreduce(id, r) to the "master" (W:276)
        return out

    def prefers_lane_output(self) -> bool:
        """Calls without ``out`` skip a copy on this lane: the one-sided lane
        with ``onesided_options={"window_output": True}`` returns its window
        row (valid until the next call) instead of writing a caller buffer."""
        return bool(self._lane_os and self._exact_os is not None and self._exact_os.window_output)

    def runs_async(self) -> bool:
        """Whether the DDP hook should issue ``async_op=True`` rounds (then
        ``async_stream()`` is where their results complete).  Not on the
        one-sided lane with its full grid: its round keeps a wave on every
        SIMD while it waits for peers, so the backward kernels an async round
        would overlap wait for it anyway, and the side-stream hand-offs cost
        more than they save (bench/ddp_overlap.py, 2 ranks: 3.11 ms per DDP
        step sync vs 4.57 async; profiles/r04/README.md).  Yes with a bounded
        footprint on a GPU of its own (``onesided_options={"cu_keep": k}``):
        the round then holds k of every 8 CUs and the backward runs on the
        rest.  Not on the direct ipc lanes (full grid, caller's stream)."""
        if self.transport == "onesided":  # (paced calls wait for their round on the caller's side)
            return self.pacer is None and self._os.bounded_footprint
        if self._lane_os:
            return self._exact_os.bounded_footprint
        if getattr(self, "_ipc_direct", False):
            return False
        return self.transport == "stream"

    def async_stream(self):
        """The stream an async round's result completes on (see runs_async)."""
        if self.transport == "onesided":
            return self._os._side_stream()
        if self._lane_os:
            return self._exact_os._side_stream()
        return self.worker._internal_streams()[1]

    def set_lane(self, lane: str) -> None:
        """Switch the exact-round lane (``auto`` / ``p2p`` / ``collective``,
        csrc/transport/stream_link.h) -- every rank must switch at the same round."""
        if self.transport != "stream":
            raise ValueError("lanes belong to the scheduled (stream) transport")
        self._lane_os = False
        self._ipc_direct_off()
        self.worker.set_lane(lane)

    def _ipc_direct_off(self) -> None:
        """Back from direct ipc rounds: the lane's round id returns to the host
        (every rank at the same round, like any lane switch)."""
        if getattr(self, "_ipc_dev_on", False):
            torch.cuda.synchronize(self.device)
            self.worker._core.ipc_device_rounds(False)
            self._ipc_dev_on = False
        self._ipc_direct = False

    def _ipc_direct_round(self, x: torch.Tensor, out: Optional[torch.Tensor]) -> AllReduceOutput:
        core = self.worker._core
        if not getattr(self, "_ipc_dev_on", False):
            core.ipc_device_rounds(True)  # collective in effect: every rank switches at the same round
            self._ipc_dev_on = True
        g = self.worker.geometry
        if getattr(self, "_full_counts", None) is None:
            self._full_counts = torch.full((g.workerNum, g.kmax), g.workerNum, dtype=torch.int32, device=self.device)
        if x.dtype != self.worker.dtype or not x.is_contiguous() or x.device != self.device:
            x = x.to(device=self.device, dtype=self.worker.dtype).contiguous()
        if out is None:
            out = torch.empty_like(x)
        # (raises once an earlier round's wait failed; a failing round zeroes
        # the fixed counts table on the device, so no output of a dead lane
        # reads as exact)
        core.ipc_round_direct(x.data_ptr(), out.data_ptr(), _raw_stream(self.device.index),
                              self._full_counts.data_ptr(), self._full_counts.numel(), self._ipc_finish)
        return AllReduceOutput(out.view(-1), iteration=self._round, counts_per_chunk=self._full_counts, geometry=g,
                               expander=self.worker._expand_counts)

    def enable_ipc(self) -> None:
        """Open the one-sided xGMI lane (csrc/transport/ipc_lane.h): every
        rank creates its window, the handles go to every rank (the TCPStore
        given at construction, else torch.distributed), every rank maps the
        others'.  Collective; afterwards ``set_lane("ipc")`` runs exact rounds
        as push / reduce / pull kernels over mapped peer memory."""
        if self.transport != "stream" or self.device.type != "cuda" or self.world_size < 2:
            raise ValueError("the ipc lane needs the stream transport on GPUs with N > 1")
        # every rank takes part in the exchange even if its own window failed
        # (an empty handle), so a local failure can never leave the others
        # blocked in the collective
        err = None
        try:
            # windows sized for ipc_capacity; an engine sharing another's
            # transport reuses that engine's windows when they fit (IpcLane)
            share = self._share.worker if (self._share is not None and self._share.worker is not None) else None
            mine = self.worker.ipc_handle(self._ipc_capacity, share)
        except Exception as e:  # noqa: BLE001 - re-raised below, after the exchange
            mine, err = b"", e
        if self.store is not None:
            self._ipc_epoch += 1
            key = f"akka/ipc/{self._iid}/{self._ipc_epoch}"
            self.store.set(f"{key}/{self.rank}", mine)
            handles = [bytes(self.store.get(f"{key}/{i}")) for i in range(self.world_size)]
        else:
            import torch.distributed as dist

            if not dist.is_initialized():
                raise RuntimeError("enable_ipc: initialise torch.distributed (gloo is enough) or pass a store")
            handles = [None] * self.world_size
            dist.all_gather_object(handles, mine)
        if err is not None:
            raise err
        missing = [i for i, h in enumerate(handles) if not h]
        if missing:
            raise RuntimeError(f"enable_ipc: ranks {missing} could not create their ipc windows")
        t0 = time.perf_counter()
        self.worker.ipc_open(handles)
        self.ipc_open_s = time.perf_counter() - t0  # mapping the peers' windows (no rendezvous in it)

    def set_ipc_mode(self, mode: str, fused: bool = False, threads: int = 0, lite: Optional[bool] = None) -> None:
        """Phase 2 of the ipc lane: ``"pull"`` or ``"bcast"``, optionally ``fused``
        into one launch, with ``threads`` per workgroup, ``lite`` fence-free
        hand-offs (AllreduceWorker.ipc_set_mode)."""
        self.worker.ipc_set_mode(mode, fused, threads, lite)

    def ipc_error(self) -> int:
        """Non-zero once a wait of the ipc lane timed out (synchronises)."""
        return self.worker.ipc_error()

    def set_exact_unit_bytes(self, nbytes: int = -1) -> None:
        """Transfer-unit size of exact p2p-lane rounds (AllreduceWorker.set_exact_unit_bytes)."""
        if self.transport != "stream":
            raise ValueError("transfer units belong to the scheduled (stream) transport")
        self.worker.set_exact_unit_bytes(nbytes)

    def set_graphs(self, on: bool = True) -> None:
        """HIP-graph replay of exact p2p-lane rounds (see AllreduceWorker.set_graphs)."""
        if self.transport != "stream":
            raise ValueError("graphs belong to the scheduled (stream) transport")
        self.worker.set_graphs(on)

    # ---- lane tuning -------------------------------------------------------
    LANES = {  # candidate -> (lane, exact transfer-unit bytes or -1, ipc mode, ipc fused, ipc workgroup size, lite)
        # RCCL's own reduce-scatter + all-gather: the comparator, never chosen by tune()
        "collective": ("collective", -1, None, False, 0, False),
        # the chunk-pipelined p2p schedule (RCCL send/recv + the gfx950 reduce)
        "p2p": ("p2p", -1, None, False, 0, False),
        # the ipc round through the engine's bookkeeping: the exact lane of
        # paced jobs (thAllreduce pacing needs the engine's round ids); its
        # safe alternative there is p2p
        "ipc_fused_lite": ("ipc", -1, "pull", True, 1024, True),
        # ipc rounds launched straight on the caller's stream with a
        # device-resident round id (no engine bookkeeping, no cross-stream
        # events; exact rounds only -- every count is N): fence-free
        # hand-offs (write-through window stores, system-coherent loads),
        # unfused and fused ...
        "ipc_lite_direct": ("ipc", -1, "pull", False, 1024, True),
        "ipc_fused_lite_direct": ("ipc", -1, "pull", True, 1024, True),
        # ... and their FENCED twin: plain window stores behind system release /
        # acquire fences (the HIP memory model's protocol), for a link on which
        # write-through + drain is not proven (or fails tune()'s validation burst)
        "ipc_fused_direct": ("ipc", -1, "pull", True, 1024, False),
        # the one-sided threshold lane at thresholds 1 (enable_onesided): one
        # role-partitioned launch, each chunk reduced and pushed as soon as
        # its copies landed, peer chunks copied out as they land; lite and fenced
        "onesided": ("onesided", -1, None, False, 0, False),
        "onesided_fenced": ("onesided", -1, None, False, 0, True),
    }

    BURST_ROUNDS = 32  # tune(): back-to-back validation rounds every candidate must pass

    @staticmethod
    def lane_candidates(*, two_sided: bool, ipc_open: bool, onesided_ok: bool, exact: bool = True,
                        paced: bool = False) -> list:
        """The lanes tune() tries (every entry of LANES but the comparator):
        the p2p schedule (RCCL p2p + the gfx950 reduce), the direct ipc rounds
        (lite, fused lite, and the fused round's FENCED twin) and the one-sided
        lane in both hand-off modes -- each fast lite lane next to a fenced
        one, so a job on a node it has never run on never depends on an
        unproven hand-off.  Paced jobs cannot take direct rounds: the
        engine-path fused ipc round stands in (p2p is its safe alternative)."""
        c: list = []
        if two_sided:
            c.append("p2p")
        if ipc_open:
            c += ["ipc_lite_direct", "ipc_fused_lite_direct", "ipc_fused_direct"] if exact and not paced \
                else ["ipc_fused_lite"]
        if onesided_ok and exact:
            c += ["onesided", "onesided_fenced"]
        return c

    def capturable(self) -> "CapturableExact":
        """A graph-capturable view of this engine's exact rounds (GPU, N > 1):
        the one-sided lane (lane ``"onesided"``) or the ipc lane with its
        round id moved to device memory.  Its calls launch the lane's kernels
        straight on the caller's stream with fixed arguments (give ``out``),
        so ``GraphedDPStep(allreduce=..., lr=...)`` can capture a whole
        training step.  Collective (every rank, same round); while it is open
        the engine's own calls are refused (``close()`` returns to them)."""
        return CapturableExact(self)

    def enable_onesided(self) -> None:
        """Map the one-sided threshold lane (parallel/onesided.py) for this
        buffer at thresholds 1: exact rounds as the lane's role-partitioned
        launch (per-chunk reduce + push the moment a chunk's copies landed).
        Collective, like enable_ipc."""
        if self._exact_os is not None:
            return
        if self.world_size < 2:
            raise ValueError("the onesided lane needs N > 1")
        if not self._th_exact:
            raise ValueError("lane 'onesided' of this engine runs exact rounds (thresholds 1); use "
                             "transport='onesided' for threshold rounds")
        from .onesided import OneSidedAllreduce

        g = self.worker.geometry
        # exact rounds take milliseconds: a 10 s bound ends a misbehaving
        # lane's waits (forced, error flagged -> rejected by tune) well inside
        # a job's phase deadlines
        self._exact_os = OneSidedAllreduce(self.data_size, max_chunk_size=int(g.maxChunkSize), dtype=self.worker.dtype,
                                           th_reduce=1.0, th_complete=1.0, max_lag=1, rank=self.rank,
                                           world_size=self.world_size, device=self.device, store=self.store,
                                           **{"timeout_s": 10.0, **self.onesided_options})

    def use_lane(self, name: str) -> None:
        """Switch to a named lane candidate (see LANES); every rank must do the
        same at the same round."""
        if name in ("onesided", "onesided_fenced"):
            self._ipc_direct_off()
            self.enable_onesided()
            self._exact_os.set_handoff("fenced" if name == "onesided_fenced" else "lite")
            self._lane_os = True
            return
        self._lane_os = False
        ln, unit, mode, fused, threads, lite = self.LANES[name]
        if name.endswith("_direct"):
            if not self._th_exact or self.device.type != "cuda" or self.world_size < 2 or self.pacer is not None:
                raise ValueError("direct ipc rounds are exact, unpaced, on GPUs with N > 1")
        else:
            self._ipc_direct_off()
        self.set_lane(ln)
        if ln == "ipc":
            self.set_ipc_mode(mode, fused, threads, lite)
        elif self.world_size > 1:
            self.set_exact_unit_bytes(unit)
        self._ipc_direct = name.endswith("_direct")

    def tune(self, candidates=None, rounds: int = 8, try_ipc: bool = True) -> dict:
        """Pick the fastest exact lane for this buffer on this job (collective).

        Every candidate runs three exact rounds with different integer data (the
        last after `rounds` timed rounds of other data, so a stale read shows),
        the timed rounds, and a validation burst of BURST_ROUNDS back-to-back
        rounds with distinct per-rank, per-round data compared on the device:
        one wrong element in any round on any rank disqualifies it (a fast
        lite lane then loses to its fenced twin).  Each step runs inside a try and is agreed on
        (max over ranks of failure and time) before the next: a step that
        fails on any rank ends the candidate on every rank.  The
        one-sided lanes join when every rank could map every other rank's
        window.  Leaves the object on the winner; returns every candidate's
        result and the choice.  Needs thresholds 1 (exact rounds)."""
        import time

        import torch.distributed as dist

        if self.transport != "stream" or self.world_size < 2:
            raise ValueError("lane tuning needs the stream transport and N > 1")
        res: dict = {}
        os_made_here = False  # tune() mapped the one-sided lane (and may drop it again)
        ipc_open = bool(self.state().get("link", {}).get("ipc"))
        cands = list(candidates) if candidates is not None else None
        if cands is None:
            spec = self.worker.transport_spec or ("",)
            # framework lanes only: the p2p schedule (gfx950 reduce) and the
            # one-sided ipc kernels.  RCCL's own reduce-scatter + all-gather
            # ("collective") is a comparator, never a candidate.  "none": ipc-only job
            os_ok = False
            if self.device.type == "cuda" and try_ipc:
                if not ipc_open:
                    err = None
                    try:
                        self.enable_ipc()
                    except Exception as e:  # noqa: BLE001 - the ipc lanes are skipped
                        err = f"{type(e).__name__}: {e}"[:200]
                    ipc_open = self._agree_max([1.0 if err else 0.0])[0] == 0.0
                    if not ipc_open:
                        res["ipc"] = {"exact": None, "ms": None,
                                      "error": err or "another rank could not open its windows"}
                if self._th_exact:
                    err = None
                    os_made_here = self._exact_os is None
                    try:
                        self.enable_onesided()
                    except Exception as e:  # noqa: BLE001 - the candidate is skipped on every rank
                        err = f"{type(e).__name__}: {e}"[:200]
                    if self._agree_max([1.0 if err else 0.0])[0] == 0.0:
                        os_ok = True
                    else:
                        res["onesided"] = {"exact": None, "ms": None,
                                           "error": err or "another rank could not map its one-sided windows"}
            cands = self.lane_candidates(two_sided=spec[0] != "none",
                                         ipc_open=ipc_open and self.device.type == "cuda" and try_ipc,
                                         onesided_ok=os_ok, exact=self._th_exact, paced=self.pacer is not None)
        S, N, r = self.data_size, self.world_size, self.rank
        dtype = self.worker.dtype
        x = torch.randn(S, device=self.device).to(dtype)
        buf = torch.empty(S, device=self.device, dtype=dtype)
        cuda = self.device.type == "cuda"

        def sync():
            if cuda:
                torch.cuda.synchronize(self.device)

        def exact(salt: int) -> bool:
            y = torch.full((S,), float((r + 1) * (salt + 1)), device=self.device, dtype=dtype)
            o = self(y)
            want = float((salt + 1) * N * (N + 1) // 2)
            return bool(torch.all(o.data == want).item()) and bool(torch.all(o.count == N).item())

        # Validation burst (first contact with a node, docs/DESIGN.md 4f rule 4):
        # BURST_ROUNDS back-to-back rounds, no host sync in between, every
        # rank's input distinct per round -- (rank + 1) * 2^(k % 8) times a
        # 1 / 2 pattern that flips every 61 elements -- and every output
        # compared on the device with its exact sum (integers of at most
        # 9 bits times a power of two: exact in fp32 and bf16 for N <= 16).
        # A stale, torn or misplaced chunk in any round makes it non-zero.
        pattern = (1 + (torch.arange(S, device=self.device) // 61) % 2).to(dtype)
        tot = N * (N + 1) // 2

        def burst(name: str) -> int:
            from ..utils.faults import env_corrupt_round

            hit = env_corrupt_round(r, name)
            xin = torch.empty(S, device=self.device, dtype=dtype)
            want = torch.empty(S, device=self.device, dtype=dtype)
            bad = torch.zeros((), dtype=torch.int64, device=self.device)
            for k in range(self.BURST_ROUNDS):
                sc = float(1 << (k % 8))
                torch.mul(pattern, (r + 1) * sc, out=xin)
                o = self(xin, out=None if self.prefers_lane_output() else buf)
                d = o.data.view(-1)
                if k == hit and S > 0:
                    d[(k * 7919) % S] += 1  # injected fault: one element of one round on this rank
                torch.mul(pattern, tot * sc, out=want)
                bad += torch.ne(d, want).sum()
            return int(bad.item())

        def timed_block() -> float:
            ob = None if self.prefers_lane_output() else buf  # the lane's own output where it has one
            o = self(x, async_op=cuda, out=ob)
            o.wait()
            sync()
            best = float("inf")
            for _ in range(2):  # the better of two blocks: one noisy block does not decide the lane
                t0 = time.perf_counter()
                for _ in range(rounds):  # the ranks are coupled by the rounds themselves
                    o = self(x, async_op=cuda, out=ob)
                o.wait()
                sync()
                best = min(best, (time.perf_counter() - t0) / rounds * 1e3)
            return best

        for name in cands:
            ok, ms, err = True, 0.0, None
            # Every step is agreed on before the next one runs: a step that
            # raised on one rank only ends the candidate on EVERY rank, so no
            # rank issues rounds its peers will never match (p2p lanes).
            steps = [("lane", lambda: (self.use_lane(name), True)[1]), ("exact1", lambda: exact(1)),
                     ("exact2", lambda: exact(2)), ("timed", timed_block), ("exact3", lambda: exact(3)),
                     ("burst", lambda: burst(name))]
            burst_bad = None
            for tag, step in steps:
                val = 0.0
                try:
                    v = step()
                    if tag in ("timed", "burst"):
                        val = float(v)
                        if tag == "burst" and v:
                            ok, err = False, f"burst: {int(v)} wrong elements on this rank"
                    elif not v:
                        ok = False
                    if name.startswith("onesided") and self._exact_os is not None and self._exact_os.error():
                        ok, err = False, f"{tag}: a bounded wait of the onesided lane expired"
                except Exception as e:  # noqa: BLE001 - the candidate is rejected
                    ok, err = False, f"{tag}: {type(e).__name__}: {e}"[:160]
                bad, worst = self._agree_max([0.0 if ok else 1.0, val])
                if tag == "timed":
                    ms = worst
                elif tag == "burst":
                    burst_bad = int(worst)  # the worst rank's count
                if bad != 0.0:
                    ok = False
                    break
            res[name] = {"exact": ok, "ms": round(ms, 4) if ok else None}
            if burst_bad is not None:
                res[name]["burst"] = {"rounds": self.BURST_ROUNDS, "bad_elements_max_rank": burst_bad}
            if err:
                res[name]["error"] = err
        good = [n for n in cands if res[n]["exact"]]
        if not good:
            raise RuntimeError(f"no exact lane: {res}")
        pick = min(good, key=lambda n: res[n]["ms"])
        if not pick.startswith("onesided") and os_made_here and self._exact_os is not None:
            # the one-sided windows (2 x rows x the buffer) are not kept for
            # a lane that lost: every rank is past its last round on them
            # (the agreement below is the barrier), then each frees its own
            if cuda:
                torch.cuda.synchronize(self.device)
            self._agree_max([0.0])
            self._exact_os = None
        self.use_lane(pick)
        res["chosen"] = pick
        self.tuned = res
        return res

    def _agree_max(self, vals: list) -> list:
        """Element-wise max over ranks of a few floats.  Over the job's store
        when one was given; else over torch.distributed with a tensor the
        default group's backend can reduce (a CUDA tensor for nccl = RCCL,
        which has no CPU path; a CPU tensor for gloo)."""
        import json

        vals = [float(v) for v in vals]
        if self.world_size < 2:
            return vals
        if self.store is not None:
            seq = getattr(self, "_agree_seq", 0)
            self._agree_seq = seq + 1
            key = f"akka/agree/{self._iid}/{seq}"
            self.store.set(f"{key}/{self.rank}", json.dumps(vals))
            rows = [json.loads(bytes(self.store.get(f"{key}/{i}")).decode()) for i in range(self.world_size)]
            return [max(r[j] for r in rows) for j in range(len(vals))]
        import torch.distributed as dist

        dev = self.device if (dist.get_backend() == "nccl" and self.device.type == "cuda") else torch.device("cpu")
        t = torch.tensor(vals, dtype=torch.float64 if dev.type == "cpu" else torch.float32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t.cpu().tolist()]

    def state(self) -> dict:
        if self._lane_os:
            st = self.worker.state()
            link = dict(st.get("link", {}))
            link["lane"] = "onesided_fenced" if self._exact_os.handoff == "fenced" else "onesided"
            link["onesided"] = {**self._exact_os.info(), "stats": self._exact_os.stats()}
            return {**st, "link": link}
        if self.transport == "onesided":
            return {"link": {"lane": "onesided", "onesided": {**self._os.info(), "stats": self._os.stats()}},
                    "stats": {"rounds_forced": self._os.stats()["complete_forced"]}}
        return self.worker.state()

    def retire(self) -> None:
        """Onesided transport: this rank serves no further round (the job's end)."""
        if self.transport == "onesided":
            self._os.retire()

    def synchronize(self) -> None:
        """Drain the reactive transport's in-flight transfers, then wait for
        this rank's queued device work."""
        if self.transport == "onesided":
            self._os.synchronize()
            return
        self.drain()
        self.worker.synchronize()

    def drain(self, timeout: float = 60.0) -> None:
        """Reactive transport: keep driving until none of this rank's transfers
        is in flight (slow peers caught up).  Call before tearing down and
        before any other blocking collective: on CPU processes (gloo) a rank's
        sends are posted only while it polls, so a rank parked in a barrier
        would stall a peer that still needs its data.  (GPU streams progress
        on their own; there it only bounds the in-flight work.)"""
        import time

        if self.transport == "onesided":
            return  # nothing in flight between calls: every send completed inside its call
        core = self.worker._core
        if not core.reactive():
            return
        t0 = time.monotonic()
        while core.in_flight():
            if not self.worker.poll():
                time.sleep(1e-4)
            if time.monotonic() - t0 > timeout:
                raise TimeoutError(f"rank {self.rank}: {core.in_flight()} transfers still in flight")


class CapturableExact:
    """Exact rounds of a ``ThresholdAllreduce`` as a capturable callable
    (``ThresholdAllreduce.capturable()``).  Two lanes:

    * ``onesided``: the engine's one-sided lane (its call id, round and
      decisions are device-resident by design);
    * ``ipc``: the engine's ipc lane with DEVICE rounds -- a bump launch
      advances a device round word in front of every round and the round's
      kernels read their id there (csrc/kernels/ipc_kernels.h ``round_dev``),
      so a captured round replays with a fresh id on every rank.
    The counts of an exact round are N everywhere (a fixed table)."""

    def __init__(self, ar: "ThresholdAllreduce"):
        if ar.transport != "stream" or ar.world_size < 2 or ar.device.type != "cuda":
            raise ValueError("capturable rounds need the stream transport on GPUs with N > 1")
        if not ar._th_exact:
            raise ValueError("capturable rounds are exact (thresholds 1)")
        self.ar = ar
        g = ar.worker.geometry
        self.geometry = g
        if ar._lane_os:
            self.lane = "onesided"
        elif ar.state().get("link", {}).get("ipc"):
            self.lane = "ipc"
            ar.worker._core.ipc_device_rounds(True)  # collective in effect: same round on every rank
            ar._ipc_dev_on = True
            self.counts = torch.full((g.workerNum, g.kmax), g.workerNum, dtype=torch.int32, device=ar.device)
        else:
            raise ValueError("capturable rounds run on the ipc or onesided lane: use_lane() one of them first")
        ar._direct = self

    @property
    def capturable(self) -> bool:
        return True

    def note_replays(self, n: int) -> None:
        if self.lane == "onesided":
            self.ar._exact_os.note_replays(n)
        elif self.ar.worker._core.ipc_error_now():
            # a replayed round's wait failed (the fixed counts table now reads
            # 0): the lane is dead, like the engine path's next round
            raise RuntimeError("ipc lane: a wait of a replayed round timed out (peer missing?); "
                               "its rounds are not trustworthy")

    def __call__(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> AllReduceOutput:
        if self.lane == "onesided":
            return self.ar._exact_os(x, out=out)
        g = self.geometry
        if out is None:
            out = torch.empty_like(x)
        self.ar.worker._core.ipc_round_direct(x.data_ptr(), out.data_ptr(), _raw_stream(self.ar.device.index),
                                              self.counts.data_ptr(), self.counts.numel())
        return AllReduceOutput(out, iteration=-1, counts_per_chunk=self.counts, geometry=g,
                               expander=self.ar.worker._expand_counts)

    def close(self) -> None:
        """Back to the engine's own calls (every rank, same round)."""
        if self.lane == "ipc" and not getattr(self.ar, "_ipc_direct", False):
            self.ar.worker._core.ipc_device_rounds(False)
            self.ar._ipc_dev_on = False
        self.ar._direct = None
