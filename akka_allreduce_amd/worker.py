"""AllreduceWorker: one per rank (reference ``AllreduceWorker.scala:7-363``).

The worker is an actor-style object: ``tell(msg)`` / ``receive(msg)`` accept
the reference's messages (``InitWorkers``, ``StartAllreduce``, ``ScatterBlock``,
``ReduceBlock``) plus ``WorkerTerminated``.  All round/threshold logic runs in
the native engine (``csrc/engine/engine.cpp``); this class owns the round
memory (torch tensors), calls the user's data source/sink, and routes outgoing
messages to peer references.

Transports
----------
``outbox``  every outgoing ScatterBlock/ReduceBlock is materialised as a message
            and handed to the destination reference's ``tell`` (the TestKit
            probe in the spec tests, a TCP proxy in a CPU cluster, an in-process
            mailbox in the local actor system).
``stream``  production: sends/receives are RCCL p2p groups over xGMI scheduled
            by the native StreamLink; no per-chunk Python work at all.  Also
            runs on the CPU p2p simulator (``transport_spec=("sim", hub, rank)``).

Every handler is wrapped like the reference's ``tryCatch`` (W:287-299): errors
are logged and recorded in ``errors`` and the worker keeps going, unless
``strict=True``.
"""
from __future__ import annotations

import logging
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from .data import AllReduceInput, AllReduceInputRequest, AllReduceOutput, Geometry
from .utils import tracing as _tracing
from .messages import (
    CompleteAllreduce,
    InitWorkers,
    ReduceBlock,
    ScatterBlock,
    StartAllreduce,
    WorkerTerminated,
)

log = logging.getLogger("akka_allreduce_amd.worker")

DataSource = Callable[[AllReduceInputRequest], AllReduceInput]
DataSink = Callable[[AllReduceOutput], None]

_DTYPES = {torch.float32: "float32", torch.bfloat16: "bfloat16"}


def _raw_stream(index: int) -> int:
    """The current stream of device ``index`` as a raw handle: ~0.1 us, where
    ``torch.cuda.current_stream(dev).cuda_stream`` builds a Stream object
    (~1.7 us, a sixth of a small round's host time on MI355X)."""
    return torch._C._cuda_getCurrentRawStream(index)


if not hasattr(torch._C, "_cuda_getCurrentRawStream"):  # pragma: no cover - older torch builds
    def _raw_stream(index: int) -> int:  # noqa: F811
        return torch.cuda.current_stream(index).cuda_stream


def _native():
    from . import _native_loader

    return _native_loader.load()


def _resolve_device(device: Any) -> torch.device:
    if device is None or device == "cpu":
        return torch.device("cpu")
    if device == "auto":
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class AllreduceWorker:
    """Threshold-allreduce worker (one per GPU rank, or per CPU process)."""

    def __init__(
        self,
        dataSource: Optional[DataSource] = None,
        dataSink: Optional[DataSink] = None,
        *,
        device: Any = None,
        dtype: torch.dtype = torch.float32,
        transport: str = "outbox",
        transport_spec: Optional[Tuple[Any, ...]] = None,
        broadcast_lag: int = 2,
        strict: bool = False,
        name: str = "worker",
    ):
        if dtype not in _DTYPES:
            raise ValueError(f"unsupported dtype {dtype}; use float32 or bfloat16")
        self.dataSource = dataSource if dataSource is not None else self._feed_source
        self.dataSink = dataSink
        self.device = _resolve_device(device)
        self.dtype = dtype
        self.transport = transport
        self.transport_spec = transport_spec
        self.strict = strict
        self.name = name
        n = _native()
        # host streams are queues this process runs: the simulator steps them,
        # async-callback (gloo) workers step them in poll()
        deferred = bool(transport_spec and transport_spec[0] in ("sim", "async_callback"))
        if transport_spec and transport_spec[0] == "shared":
            deferred = transport_spec[1]._deferred  # the adopted device's kind
        self._deferred = deferred
        dev_index = self.device.index if self.device.type == "cuda" else -1
        self._core = n.WorkerCore(self, transport, dev_index, _DTYPES[dtype], deferred, broadcast_lag)
        self.id: int = -1
        self.peers: Dict[int, Any] = {}
        self.master: Any = None
        self.geometry: Optional[Geometry] = None
        self.errors: List[BaseException] = []
        self._rounds: Dict[int, Dict[str, torch.Tensor]] = {}
        self._pre_init: List[Any] = []
        self._to_release: List[int] = []
        self._feed: Dict[int, torch.Tensor] = {}
        self._outputs: Dict[int, AllReduceOutput] = {}
        self._next_round = 0
        self._in_call = 0
        self._frames_ok: Optional[bool] = None  # every peer takes wire frames (see _flush_outbox)
        self._stream_cache: Optional[int] = None
        # CPU race checking (AKKA_RACECHECK=1): a stream of the simulated
        # device standing for the caller's stream (producer of inputs,
        # allocator of outputs); see csrc/engine/racecheck.h
        self.host_stream: Optional[int] = None
        self._async = False
        self._ext_streams = None
        self._out_override: Dict[int, torch.Tensor] = {}
        self._delivered: set = set()
        self._core_reactive = transport == "reactive"
        self._fast_source = dataSource is None  # rounds fed by allreduce(): eligible for the native fast path
        self._fast_pending: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        self.fast_rounds = 0  # rounds that took the native fast path
        self._cuda = self.device.type == "cuda"
        self._dev_index = self.device.index if self._cuda else -1
        self._counts_by_out: Dict[int, torch.Tensor] = {}
        self.epochs = 0  # RCCL membership epochs after the first (re-InitWorkers with a new unique id)
        self.reactive_timeout: Optional[float] = None  # reactive allreduce(): max seconds to wait

    @staticmethod
    def startUp(port: int, dataSize: int, checkpoint: int = 50, assertMultiple: int = 0,
                master: Optional[str] = None, **kw):
        """Reference entry point ``AllreduceWorker.startUp(port, dataSize,
        checkpoint, assertMultiple)`` (W:348-362): a worker process joining the
        master (default: the configured seed node, CONF:13-16) with the demo
        data source and throughput/exactness sink.  Returns the ``WorkerProcess``."""
        from .config import load_config
        from .parallel.cluster import start_worker

        if master is None:
            cfg = load_config(None)
            master = f"{cfg.cluster.host}:{cfg.cluster.port}"
        return start_worker(master, int(dataSize), checkpoint=int(checkpoint), assert_multiple=int(assertMultiple),
                            port=int(port), **kw)

    # ------------------------------------------------------------------ actor API
    def tell(self, msg: Any, sender: Any = None) -> None:
        self.receive(msg)

    def receive(self, msg: Any) -> None:
        self._in_call += 1
        try:
            self._dispatch(msg)
        except Exception as e:  # tryCatch: log and keep the worker alive (W:287-299)
            self.errors.append(e)
            log.error("%s: error handling %s: %s", self.name, type(msg).__name__, e)
            if self.strict:
                raise
        finally:
            self._in_call -= 1
            if self._in_call == 0:
                self._flush_outbox()
                self._release_pending()

    def consume_frames(self, splitter: Any, deliver: Callable[[bytes], None]) -> None:
        """The frames one ``recv`` completed (the actor runtime's native path,
        Node.frame_consumer): the native splitter applies every ScatterBlock /
        ReduceBlock of this worker's dtype in C++ with a pointer into the
        frame; any other frame -- or every frame while the worker is not
        initialized on the message-driven (TCP) data plane -- comes back in
        order and goes to ``deliver`` (decode + ``receive``).  Sends are held
        until the end, so the replies to a burst of chunks leave as one write
        per peer."""
        self._in_call += 1
        try:
            while True:
                core = self._core
                ok = core is not None and self.initialized and not self._pre_init and self.transport == "outbox"
                try:
                    body = splitter.run(core if ok else None)
                except ValueError:
                    raise  # a corrupt stream: the runtime closes the connection
                except Exception as e:  # the frame is consumed; tryCatch semantics (W:287-299)
                    self.errors.append(e)
                    log.error("%s: error handling a data frame: %s", self.name, e)
                    if self.strict:
                        raise
                    continue
                if body is None:
                    return
                deliver(body)
        finally:
            self._in_call -= 1
            if self._in_call == 0 and self._core is not None:
                self._flush_outbox()
                self._release_pending()

    def _dispatch(self, msg: Any) -> None:
        if isinstance(msg, InitWorkers):
            self._on_init(msg)
        elif isinstance(msg, StartAllreduce):
            if not self.initialized:
                self._pre_init.append(msg)
            else:
                self._core.start(int(msg.round))
        elif isinstance(msg, ScatterBlock):
            if not self.initialized:
                self._pre_init.append(msg)
                return
            t = self._payload(msg.value)
            self._core.scatter_in(int(msg.srcId), int(msg.destId), int(msg.chunkId), int(msg.round),
                                  t.data_ptr(), t.numel(), t.device.type == "cpu")
            self._sync_if_device_payload(t)
        elif isinstance(msg, ReduceBlock):
            if not self.initialized:
                self._pre_init.append(msg)
                return
            t = self._payload(msg.value)
            self._core.reduce_in(int(msg.srcId), int(msg.destId), int(msg.chunkId), int(msg.round), int(msg.count),
                                 t.data_ptr(), t.numel(), t.device.type == "cpu")
            self._sync_if_device_payload(t)
        elif isinstance(msg, WorkerTerminated):
            self.peers.pop(int(msg.workerId), None)
            if self.initialized:
                self._core.peer_terminated(int(msg.workerId))
        else:
            raise TypeError(f"unhandled message {msg!r}")

    def _on_init(self, m: InitWorkers) -> None:
        # a reference to this worker itself (or a local wrapper of it) short-circuits (W:228)
        peers = [(int(i), ref is self or getattr(ref, "actor", None) is self) for i, ref in m.workers.items()]
        tinfo = getattr(m, "transport", None)
        rccl = bool(tinfo and tinfo.get("kind") == "rccl" and self.transport in ("stream", "reactive"))
        if rccl and self.transport_spec is None:
            self.transport_spec = ("rccl", tinfo["uid"], int(m.destId), int(m.workerNum),
                                   list(tinfo.get("members") or []))
        elif tinfo and tinfo.get("kind") == "ipc_p2p" and self.transport_spec is None \
                and self.transport in ("stream", "reactive"):
            # mailboxes in mapped peer memory; handles meet in the master's store
            from torch.distributed import TCPStore

            from .parallel.collective import _handle_exchange

            host, port = tinfo["store"]
            store = TCPStore(host, int(port), is_master=False)
            self._ipc_store = store  # keep the connection for the job's lifetime
            self.transport_spec = ("ipc_p2p", int(m.destId), int(m.workerNum),
                                   _handle_exchange(int(m.destId), int(m.workerNum), store, tinfo["key"]))
        elif tinfo and tinfo.get("kind") in ("loopback", "loopback_pair", "sim") and self.transport_spec is None:
            # in-process data planes handed out by the control plane (tests /
            # single-process clusters): the hub is shared by every worker
            self.transport_spec = (tinfo["kind"], tinfo["hub"], int(m.destId))
        if self.transport_spec and self.transport_spec[0] == "shared" and not self.initialized:
            # this engine rides on another engine's transport (device streams +
            # communicator): ThresholdAllreduce(share_transport_with=...)
            self._core.adopt_transport(self.transport_spec[1]._core)
        first = self._core.init(int(m.destId), int(m.workerNum), float(m.thReduce), float(m.thComplete),
                                int(m.maxLag), int(m.dataSize), int(m.maxChunkSize), peers)
        self.peers = dict(m.workers)
        self._frames_ok = None
        if not first:
            # re-init only replaces the peer map (W:87-89) -- and, on the RCCL
            # data plane, starts a new membership epoch: a communicator over
            # the listed members from the new unique id (after a death / join)
            if rccl and self.transport_spec and self.transport_spec[0] == "rccl" \
                    and bytes(tinfo["uid"]) != bytes(self.transport_spec[1]):
                members = sorted(int(i) for i in (tinfo.get("members") or m.workers))
                self._core.rebuild_transport(tinfo["uid"], members)
                self.transport_spec = ("rccl", tinfo["uid"], self.id, int(m.workerNum), members)
                self.epochs += 1
            return
        self.id = int(m.destId)
        self.master = m.master
        self.geometry = Geometry(int(m.dataSize), int(m.workerNum), int(m.maxChunkSize))
        self._connect_transport()
        self._core.attach()
        st = self._core.state()
        log.info("%s: id=%d peers %d/%d thReduce=%s thComplete=%s maxLag=%d scatter threshold=%d reduce threshold=%d",
                 self.name, self.id, len(self.peers), m.workerNum, m.thReduce, m.thComplete, m.maxLag,
                 st["min_scatter_required"], st["min_reduced_required"])
        pending, self._pre_init = self._pre_init, []
        for p in pending:
            self._dispatch(p)

    def _connect_transport(self) -> None:
        if self.transport not in ("stream", "reactive"):
            return
        spec = self.transport_spec or (("local",) if self.geometry.workerNum == 1 else None)
        if spec is None:
            raise RuntimeError("stream transport needs transport_spec=('rccl', uid, rank, nranks) or ('sim', hub, rank)")
        kind = spec[0]
        if kind == "rccl":
            _, uid, rank, nranks = spec[:4]
            members = [int(i) for i in spec[4]] if len(spec) > 4 and spec[4] else []
            self._core.connect_rccl(uid, int(rank), int(nranks), members)
        elif kind == "rccl_shape":
            _, rank, nranks = spec
            self._core.connect_rccl_shape(int(rank), int(nranks))
        elif kind == "sim":
            _, hub, rank = spec
            self._core.connect_sim(hub, int(rank))
        elif kind == "local":
            self._core.connect_local()
        elif kind == "loopback":
            _, hub, rank = spec
            self._core.connect_loopback(hub, int(rank))
        elif kind == "loopback_pair":
            _, hub, rank = spec
            self._core.connect_loopback_pair(hub, int(rank))
        elif kind == "async_callback":
            _, post, test, rank, nranks = spec
            self._core.connect_async_callback(post, test, int(rank), int(nranks))
        elif kind == "callback":
            _, fn, rank, nranks = spec
            self._core.connect_callback(fn, int(rank), int(nranks))
        elif kind == "ipc_p2p":  # grouped send/recv over mapped peer memory, handles exchanged by `exchange`
            _, rank, nranks, exchange = spec
            err = None
            try:
                self._core.connect_ipc_p2p(int(rank), int(nranks))
                mine = bytes(self._core.p2p_handle())
            except Exception as e:  # noqa: BLE001 - join the exchange anyway, then re-raise
                mine, err = b"", e
            handles = exchange(mine)
            if err is not None:
                raise err
            if not all(handles):
                raise RuntimeError("ipc p2p: some ranks could not create their mailboxes")
            self._core.p2p_open([bytes(h) for h in handles])
        elif kind == "none":  # ipc-only data plane: exact rounds on the one-sided lane
            _, rank, nranks = spec
            self._core.connect_none(int(rank), int(nranks))
        elif kind == "shared":  # another engine's transport (adopted before init)
            self._core.connect_adopted()
        else:
            raise ValueError(f"unknown transport spec {spec!r}")

    # ------------------------------------------------------------------ properties
    @property
    def initialized(self) -> bool:
        return self.id >= 0

    def state(self) -> Dict[str, Any]:
        return self._core.state()

    @property
    def round(self) -> int:
        return self._core.state()["round"]

    @property
    def maxRound(self) -> int:
        return self._core.state()["max_round"]

    @property
    def completed(self) -> List[int]:
        return self._core.state()["completed"]

    # ------------------------------------------------------------------ collective convenience API
    def allreduce(self, tensor: torch.Tensor, async_op: bool = False,
                  out: Optional[torch.Tensor] = None) -> Optional[AllReduceOutput]:
        """Start the next round with ``tensor`` as this worker's contribution.

        For the scheduled (RCCL) transport the round's whole schedule is
        enqueued on the GPU before this returns.  By default the returned
        output is valid in the caller's current stream order.  With
        ``async_op=True`` (torch.distributed's convention) the caller's stream
        is NOT made to wait: call ``out.wait()`` before using ``out.data``.
        Back-to-back async rounds then pipeline without a cross-stream hop per
        round; all tensors involved are ``record_stream``-ed on the internal
        streams so the caching allocator cannot recycle them early.
        Returns ``None`` if the round has not completed yet (threshold
        transports driven by messages).

        ``out``: a preallocated 1-D output of ``dataSize`` elements (like
        ``all_gather_into_tensor``).  Reusing one buffer across rounds keeps
        its lines in the 256 MiB Infinity Cache; rounds are written in stream
        order, so a buffer may be reused as soon as its previous round's result
        has been consumed in that order.
        """
        if self._fast_ok(tensor):
            return self._fast_allreduce(tensor, async_op, out)
        r = self._next_round
        self._next_round += 1
        self._feed[r] = tensor
        if out is not None:
            g = self.geometry
            if out.numel() != g.dataSize or out.dtype != self.dtype or out.device != self.device \
                    or not out.is_contiguous():
                raise ValueError("out must be a contiguous tensor of dataSize elements, worker dtype and device")
            self._out_override[r] = out
        # one stream lookup per call instead of one per callback
        self._stream_cache = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" \
            else (self.host_stream or 0)
        self._async = bool(async_op) and self.device.type == "cuda"
        try:
            with _tracing.range_(f"akka.round {r}"):
                self.receive(StartAllreduce(r))
        finally:
            self._stream_cache = None
            self._async = False
        if self._core.reactive() and r not in self._outputs and not self._core_is_sim():
            self.progress_until(r, self.reactive_timeout)
        return self._outputs.pop(r, None)

    def set_lane(self, lane: str) -> None:
        """Exact-round lane of the scheduled transport: ``"auto"`` (RCCL
        reduce-scatter + all-gather when available and the geometry is even,
        else the chunk-pipelined p2p schedule), ``"p2p"`` or ``"collective"``
        (see csrc/transport/stream_link.h).  Threshold rounds (< 1) always run
        the p2p schedule."""
        self._core.set_lane(lane)

    def set_exact_unit_bytes(self, nbytes: int = -1) -> None:
        """Minimum bytes per transfer unit of exact p2p-lane rounds (whole
        chunks; a unit larger than a block means one message per peer and
        phase).  -1 restores the default (AKKA_EXACT_UNIT_BYTES or 16 MiB).
        Every rank must switch at the same round."""
        self._core.set_exact_unit_bytes(int(nbytes))

    # ---- one-sided xGMI lane (csrc/transport/ipc_lane.h) ----
    def ipc_handle(self, capacity: int = 0, share: Optional["AllreduceWorker"] = None) -> bytes:
        """Create this rank's window (once) and return its handle, to be
        exchanged with every rank of the job (ipc_open).  ``capacity``: size
        the windows for that many elements; ``share``: an engine on the same
        (adopted) transport whose windows to reuse when large enough."""
        return bytes(self._core.ipc_handle(int(capacity), share._core if share is not None else None))

    def ipc_open(self, handles: list) -> None:
        """Map every other rank's window; ``handles[i]`` is rank i's
        ipc_handle().  Afterwards ``set_lane("ipc")`` is allowed."""
        self._core.ipc_open([bytes(h) for h in handles])

    def ipc_error(self) -> int:
        """Non-zero once a wait of the ipc lane timed out on this rank
        (synchronises the device)."""
        return int(self._core.ipc_error())

    def ipc_set_mode(self, mode: str, fused: bool = False, threads: int = 0, lite: Optional[bool] = None) -> None:
        """Phase 2 of the ipc lane: ``"pull"`` (every rank reads the reduced
        rows over xGMI) or ``"bcast"`` (each reducer writes its rows into every
        peer's window); ``fused``: the three phases as roles of one launch,
        pipelined by portion; ``threads``: workgroup size of the round's
        kernels (256 / 512 / 1024, 0 keeps it); ``lite``: fence-free hand-offs
        (write-through window stores, system-coherent loads; None keeps it).
        Every rank must switch at the same round."""
        self._core.ipc_set_mode(mode, bool(fused), int(threads), -1 if lite is None else int(bool(lite)))

    def ipc_close(self) -> None:
        self._core.ipc_close()

    def set_graphs(self, on: bool = True) -> None:
        """Replay exact p2p-lane rounds from captured HIP graphs: a round whose
        buffers (input, ring row, output) were seen before is captured once,
        later ones are one graph launch (stream_link.h).  GPU only."""
        self._core.set_graphs(bool(on))

    def _alloc_counts(self) -> torch.Tensor:
        g = self.geometry
        return torch.empty(g.workerNum * g.kmax, dtype=torch.int32, device=self.device)

    def _fast_ok(self, tensor: torch.Tensor) -> bool:
        """Collective-style call on the scheduled transport, whose rounds
        complete inside the call: buffers can be bound natively."""
        return (self.transport == "stream" and not self._deferred and self.id >= 0
                and self.dataSink is None and self._fast_source and not self._pre_init and not self._rounds
                and isinstance(tensor, torch.Tensor) and self._buffer_ok(tensor))

    def _buffer_ok(self, t: torch.Tensor) -> bool:
        """A contiguous tensor of dataSize elements of the worker's dtype on its
        device (plain int / identity compares: this runs twice per round)."""
        return (t.dtype is self.dtype and t.get_device() == self._dev_index and t.numel() == self.geometry.dataSize
                and t.is_contiguous())

    def _counts_for(self, out: torch.Tensor) -> torch.Tensor:
        """The [N, kmax] counts table that travels with a caller-owned output
        buffer: reused with THAT buffer (the caller reuses the buffer only once
        its previous round was consumed, which covers its counts too), so a
        round with ``out`` given allocates nothing."""
        key = out.data_ptr()
        c = self._counts_by_out.get(key)
        if c is None:
            if len(self._counts_by_out) >= 16:  # bounded: buffers the caller dropped
                self._counts_by_out.pop(next(iter(self._counts_by_out)))
            g = self.geometry
            c = self._counts_by_out[key] = torch.empty((g.workerNum, g.kmax), dtype=torch.int32, device=self.device)
        return c

    def _fast_allreduce(self, x: torch.Tensor, async_op: bool, out: Optional[torch.Tensor]) -> Optional[AllReduceOutput]:
        # The host cost of this call is the price of every small round (the
        # reference's regime: maxChunkSize 2, M:104): raw stream handle, no
        # allocation when ``out`` is given, one native call
        # (profiles/r06/small_rounds/README.md).
        g = self.geometry
        if out is None:
            out = torch.empty(g.dataSize, dtype=self.dtype, device=self.device)
            counts = torch.empty((g.workerNum, g.kmax), dtype=torch.int32, device=self.device)
        elif not self._buffer_ok(out):
            raise ValueError("out must be a contiguous tensor of dataSize elements, worker dtype and device")
        else:
            counts = self._counts_by_out.get(out.data_ptr())
            if counts is None:
                counts = self._counts_for(out)
        r = self._next_round
        self._next_round += 1
        cuda = self._cuda
        async_op = bool(async_op) and cuda
        if cuda:
            sptr = _raw_stream(self._dev_index)
            wait = not async_op
        else:
            sptr = self.host_stream or 0
            wait = self.host_stream is not None
        local = g.workerNum == 1  # a purely local round runs on the caller's stream
        if async_op and not local:
            # the caller's stream will not wait: keep every buffer alive until
            # the internal streams are past them
            self._keep_alive_on_internal_streams(x, out, counts)
        self._fast_pending[r] = (out, counts)
        try:
            if _tracing._enabled:
                with _tracing.range_(f"akka.round {r}"):
                    done = self._core.fast_round(r, x.data_ptr(), out.data_ptr(), counts.data_ptr(), sptr, wait)
            else:
                done = self._core.fast_round(r, x.data_ptr(), out.data_ptr(), counts.data_ptr(), sptr, wait)
        except Exception as e:  # tryCatch semantics as in receive()
            self._fast_pending.pop(r, None)
            self.errors.append(e)
            log.error("%s: error in round %d: %s", self.name, r, e)
            if self.strict:
                raise
            return None
        self.fast_rounds += 1
        expander = self._expand_counts if cuda else None
        res = None
        for d in done:
            o, c = self._fast_pending.pop(d)
            event = None
            if async_op:
                event = torch.cuda.Event()
                event.record(torch.cuda.current_stream(self.device) if local else self._internal_streams()[1])
            o = AllReduceOutput._make(o, d, c, g, expander, event)
            if d == r:
                res = o
            else:
                self._outputs[d] = o
        return res

    # ------------------------------------------------------------------ reactive transport progress
    def _core_is_sim(self) -> bool:
        return bool(self.transport_spec and self.transport_spec[0] == "sim")

    def poll(self) -> bool:
        """Reactive transport: hand completed transfers to the engine (which may
        reduce, complete and deliver rounds).  Returns True on progress."""
        self._in_call += 1
        try:
            return bool(self._core.poll())
        except Exception as e:
            self.errors.append(e)
            if self.strict:
                raise
            log.error("%s: error in poll: %s", self.name, e)
            return False
        finally:
            self._in_call -= 1
            if self._in_call == 0:
                self._flush_outbox()
                self._release_pending()

    def progress_until(self, round_: int, timeout: Optional[float] = None) -> None:
        """Poll until ``round_`` completed locally (threshold reached) or timeout."""
        import time as _time
        deadline = None if timeout is None else _time.monotonic() + timeout
        spins = 0
        while round_ not in self._delivered:
            if not self.poll():
                spins += 1
                if spins > 8:
                    # sleep until a pair stream signals (GIL released), not spin
                    self._core.wait_activity(200)
                    if spins > 64:
                        _time.sleep(0)  # CPU (gloo) transport: let other threads run
                if deadline is not None and _time.monotonic() > deadline:
                    st = self._core.state()
                    raise TimeoutError(f"{self.name}: round {round_} did not complete within {timeout}s "
                                       f"(engine round {st['round']}, stats {st['stats']}, link {st.get('link')})")
            else:
                spins = 0
        self._delivered.discard(round_)

    def _internal_streams(self):
        if self._ext_streams is None:
            comm, compute = self._core.streams()
            self._ext_streams = (torch.cuda.ExternalStream(comm, device=self.device),
                                 torch.cuda.ExternalStream(compute, device=self.device))
        return self._ext_streams

    def _keep_alive_on_internal_streams(self, *tensors: torch.Tensor) -> None:
        for s in self._internal_streams():
            for t in tensors:
                t.record_stream(s)

    def _feed_source(self, req: AllReduceInputRequest) -> AllReduceInput:
        t = self._feed.pop(req.iteration, None)
        if t is None:
            raise KeyError(f"no input fed for round {req.iteration}")
        return AllReduceInput(t)

    # ------------------------------------------------------------------ engine callbacks
    def _stream_ptr(self) -> int:
        if self.device.type != "cuda":
            return self.host_stream or 0
        if self._stream_cache is not None:
            return self._stream_cache
        return torch.cuda.current_stream(self.device).cuda_stream

    def _fetch(self, round_: int) -> None:
        inp = self.dataSource(AllReduceInputRequest(round_))
        data = inp.data if isinstance(inp, AllReduceInput) else inp
        t = torch.as_tensor(data)
        if t.numel() != self.geometry.dataSize:  # W:200-202
            raise ValueError(f"Input data size {t.numel()} is different from initialization time "
                             f"{self.geometry.dataSize}!")
        t = t.reshape(-1).to(device=self.device, dtype=self.dtype).contiguous()
        rec = self._rounds.setdefault(round_, {})
        rec["input"] = t
        if self._async:
            self._keep_alive_on_internal_streams(t)
        # (Synchronous rounds need no record_stream: the caller's stream waits
        # for the round's done event, which follows every read of the input --
        # including the reactive transport's staging copy -- and the caching
        # allocator only reuses the block in that stream's order.)
        self._core.bind_input(round_, t.data_ptr(), self._stream_ptr(), self._has_stream())

    def _has_stream(self) -> bool:
        return self.device.type == "cuda" or self.host_stream is not None

    def _new_output_buffers(self, round_: int) -> Tuple[torch.Tensor, torch.Tensor]:
        g = self.geometry
        out = self._out_override.pop(round_, None)
        if out is None:
            out = torch.empty(g.dataSize, dtype=self.dtype, device=self.device)
        # every entry the count expansion reads is written (uploaded or received)
        counts = torch.empty(g.workerNum * g.kmax, dtype=torch.int32, device=self.device)
        return out, counts

    def _alloc_output(self, round_: int) -> None:
        out, counts = self._new_output_buffers(round_)
        rec = self._rounds.setdefault(round_, {})
        rec["output"], rec["counts"] = out, counts
        if self._async:
            self._keep_alive_on_internal_streams(out, counts)
        # the caller's stream allocated them: engine streams that write them
        # wait for this point (memory the allocator recycled may still be in
        # use by earlier work on that stream)
        self._core.bind_output(round_, out.data_ptr(), counts.data_ptr(), self._stream_ptr(), self._has_stream())

    def _deliver(self, round_: int) -> None:
        rec = self._rounds[round_]
        event = None
        if self.device.type == "cuda":
            if self._async:
                # finalize() already queued the round's done point on the stream
                # that ran it: the compute stream, or the caller's own stream for
                # a purely local (N=1) round
                event = torch.cuda.Event()
                if self._core.exec_on_producer(round_):
                    event.record(torch.cuda.current_stream(self.device))
                else:
                    event.record(self._internal_streams()[1])
            else:
                self._core.stream_wait_done(round_, self._stream_ptr())
        elif self.host_stream is not None:
            # modelled caller stream (CPU race checking): the output is valid
            # in its order, like the caller's stream on a GPU
            self._core.stream_wait_done(round_, self.host_stream)
        g = self.geometry
        out = AllReduceOutput(rec["output"], iteration=round_,
                              counts_per_chunk=rec["counts"].view(g.workerNum, g.kmax), geometry=g,
                              expander=self._expand_counts if self.device.type == "cuda" else None,
                              event=event)
        self._to_release.append(round_)
        if self._core_reactive:
            self._delivered.add(round_)
            if len(self._delivered) > 4096:  # rounds nobody waited for
                self._delivered.discard(min(self._delivered))
        if self.dataSink is not None:
            self.dataSink(out)
        else:
            self._outputs[round_] = out

    def _notify_complete(self, round_: int) -> None:
        self._flush_outbox()  # keep message order: peer traffic emitted before completion goes first
        if self.master is not None:  # reference NPEs on a None master (W:276)
            self.master.tell(CompleteAllreduce(self.id, round_))

    def _release(self, round_: int) -> None:
        self._to_release.append(round_)

    def _expand_counts(self, per_chunk: torch.Tensor) -> torch.Tensor:
        out = torch.empty(self.geometry.dataSize, dtype=torch.int32, device=per_chunk.device)
        self._core.expand_counts(out.data_ptr(), per_chunk.contiguous().data_ptr(), self._stream_ptr())
        return out

    # ------------------------------------------------------------------ helpers
    def _payload(self, value: Any) -> torch.Tensor:
        if isinstance(value, torch.Tensor) and value.dtype is self.dtype and value.dim() == 1 \
                and value.device.type == "cpu" and value.is_contiguous():
            return value  # (a decoded wire payload: nothing to convert)
        t = value if isinstance(value, torch.Tensor) else torch.as_tensor(value)
        if t.dtype != self.dtype:
            t = t.to(self.dtype)
        t = t.reshape(-1)
        if t.device.type == "cuda" and self.device.type == "cpu":
            t = t.cpu()
        return t.contiguous()

    def _sync_if_device_payload(self, t: torch.Tensor) -> None:
        if t.device.type == "cuda":
            self._core.sync_all()  # the async D2D copy must finish before `t` can be freed

    def _flush_outbox(self) -> None:
        # one batch per remote destination, in emission order (per-pair FIFO,
        # as the reference's tests rely on): one write per peer per handler.
        # Peers that are all network references take the outbox as wire
        # frames built natively (no message object per chunk)
        if self._frames_ok is None:
            self._frames_ok = bool(self.peers) and all(hasattr(r, "tell_frames") for r in self.peers.values()
                                                       if r is not self)
        if self._frames_ok and self.transport == "outbox":
            for dest, frames in self._core.drain_frames():
                ref = self.peers.get(dest)
                if ref is None:
                    continue  # peer left the cluster
                if ref is self or not hasattr(ref, "tell_frames"):
                    self._frames_ok = None  # the peer map changed: look again
                    from .parallel.wire import FrameReader, decode  # noqa: PLC0415

                    for body in FrameReader().feed(frames):
                        ref.tell(decode(body, lambda a: None), self)
                    continue
                ref.tell_frames(frames)
            return
        batches: Dict[int, list] = {}
        for m in self._core.drain():
            value = torch.frombuffer(bytearray(m.data), dtype=self.dtype) if len(m.data) else torch.empty(0, dtype=self.dtype)
            if m.kind == 1:
                msg: Any = ScatterBlock(value, m.src, m.dest, m.chunk, m.round)
            else:
                msg = ReduceBlock(value, m.src, m.dest, m.chunk, m.round, m.count)
            ref = self.peers.get(m.dest)
            if ref is None:
                continue  # peer left the cluster
            if hasattr(ref, "tell_many"):
                batches.setdefault(m.dest, []).append(msg)
            else:
                ref.tell(msg, self)
        for dest, msgs in batches.items():
            self.peers[dest].tell_many(msgs)

    def _release_pending(self) -> None:
        if not self._to_release:
            return
        todo, self._to_release = self._to_release, []
        for r in todo:
            if r in self._rounds:
                self._core.unbind(r)
                del self._rounds[r]

    def close(self) -> None:
        """Release the native core (streams, buffers) now.  Freeing device
        memory synchronizes the whole GPU, so do it while no stream of this
        process is parked on a peer (e.g. after the reactive link drained)."""
        core, self._core = self._core, None
        self._rounds.clear()
        self._outputs.clear()
        del core

    def synchronize(self) -> None:
        """Block until all of this worker's queued device work is done."""
        self._core.sync_all()

    def __repr__(self) -> str:
        return f"AllreduceWorker(name={self.name!r}, id={self.id}, device={self.device}, transport={self.transport})"
