"""Master / worker processes: the reference's cluster bring-up, MI355X style.

Reference flow: master and workers are separate JVMs joining an
Akka cluster through seed nodes; the master registers workers on MemberUp,
watches them, and once ``totalWorkers`` joined sends InitWorkers and
StartAllreduce(0) (M:36-44, M:114-136, W:317-346).

Here every process hosts one ``Node`` (TCP endpoint + mailbox + dispatcher):
  * ``start_master`` -- the AllreduceMaster actor plus a failure detector
    (heartbeats; ``unreachable_after_s`` replaces Akka's phi-accrual detector +
    ``auto-down-unreachable-after = 10s``, CONF:18-20).  When every worker
    reports a GPU, the master also mints the RCCL unique id and ships it in
    InitWorkers so the data plane runs over xGMI; otherwise chunks travel as
    TCP messages (the reference's data path, CPU clusters).
  * ``start_worker`` -- an AllreduceWorker registering with the master
    (RegisterWorker replaces MemberUp + actorSelection.resolveOne, M:66-74),
    heartbeating, and stopping on Shutdown.
The demo data source/sink of the reference (constant 0..n-1 floats; a sink
that prints MBytes/sec every ``checkpoint`` rounds and optionally asserts the
output is ``assertMultiple`` x input, W:325-342) are provided as
``constant_source`` / ``throughput_sink``.
"""
from __future__ import annotations

import logging
import socket
import threading
import time
from typing import Any, Callable, Dict, Optional

import torch

from ..config import DataConfig, ThresholdConfig, WorkerConfig
from ..data import AllReduceInput, AllReduceInputRequest, AllReduceOutput
from ..master import AllreduceMaster
from ..messages import CompleteAllreduce, Heartbeat, RegisterWorker, Shutdown, WorkerTerminated
from ..worker import AllreduceWorker
from .actors import Node

log = logging.getLogger("akka_allreduce_amd.cluster")


# ---------------------------------------------------------------------------
# demo data source / sink (W:325-342)

def constant_source(data_size: int, dtype: torch.dtype = torch.float32) -> Callable[[AllReduceInputRequest], AllReduceInput]:
    floats = torch.arange(data_size, dtype=torch.float32).to(dtype)

    def source(_req: AllReduceInputRequest) -> AllReduceInput:
        return AllReduceInput(floats)

    return source


class ThroughputSink:
    """Prints algbw every ``checkpoint`` rounds; optional exactness assertion."""

    def __init__(self, data_size: int, checkpoint: int = 50, assert_multiple: int = 0, printer=print):
        self.data_size = data_size
        self.checkpoint = max(1, checkpoint)
        self.assert_multiple = assert_multiple
        self.tic = time.time()
        self.rounds = 0
        self.failures = 0
        self.last_mbps: Optional[float] = None
        self.printer = printer
        self.expected = torch.arange(data_size, dtype=torch.float64)

    def __call__(self, r: AllReduceOutput) -> None:
        self.rounds += 1
        if r.iteration % self.checkpoint == 0 and r.iteration != 0:
            if r.data.is_cuda:
                torch.cuda.current_stream(r.data.device).synchronize()
            elapsed = max(time.time() - self.tic, 1e-9)
            nbytes = r.data.numel() * r.data.element_size() * self.checkpoint
            self.last_mbps = nbytes / 1e6 / elapsed
            self.printer(f"----Data output at #{r.iteration} - {elapsed:.3f} s")
            self.printer("%2.1f Mbytes in %2.3f seconds at %4.3f MBytes/sec" % (nbytes / 1e6, elapsed, self.last_mbps))
            if self.assert_multiple > 0:
                ok_d = torch.equal(r.data.double().cpu(), self.expected * self.assert_multiple)
                ok_c = bool((r.count.cpu() == self.assert_multiple).all())
                if not (ok_d and ok_c):
                    self.failures += 1
                    self.printer(f"ASSERTION FAILED at round {r.iteration}: data ok={ok_d} counts ok={ok_c} "
                                 "(check that all thresholds are 1)")
            self.tic = time.time()


# ---------------------------------------------------------------------------
# master

class MasterProcess:
    def __init__(self, thresholds: ThresholdConfig, data: DataConfig, workers: WorkerConfig, *,
                 host: str = "127.0.0.1", port: int = 2551, heartbeat_interval_s: float = 1.0,
                 unreachable_after_s: float = 10.0, transport: str = "auto", min_workers: Optional[int] = None):
        self.node = Node(host, port, name="master")
        self.transport = transport
        self._store = None
        if transport in ("ipc_p2p", "onesided"):
            # the workers' rendezvous for their window handles: a key-value
            # store hosted by the master (no RCCL id to mint)
            from torch.distributed import TCPStore

            self._store = TCPStore(host, 0, is_master=True, wait_for_workers=False)
        self._gpu_workers: Dict[str, bool] = {}  # worker address -> has a GPU
        self.master = AllreduceMaster.from_configs(thresholds, data, workers, on_finished=self._finished,
                                                   transport_info=self._transport_info, min_workers=min_workers)
        self.unreachable_after_s = unreachable_after_s
        self.heartbeat_interval_s = heartbeat_interval_s
        self.last_seen: Dict[int, float] = {}
        self.node_metrics: Dict[int, Dict[str, Any]] = {}  # latest sample per worker (cluster metrics)
        self.finished = threading.Event()
        self._lock = threading.Lock()
        self.node.on_send_failure = self._send_failed
        self.node.aliases.append(self.master)
        self.node.start(self)
        self._fd = threading.Thread(target=self._failure_detector, name="master-fd", daemon=True)
        self._fd.start()
        log.info("master listening on %s (workers=%d, dataSize=%d, maxChunkSize=%d)", self.node.address,
                 workers.totalSize, data.dataSize, data.maxChunkSize)

    @property
    def address(self) -> str:
        return self.node.address

    def _transport_info(self) -> Optional[Dict[str, Any]]:
        if self._store is not None:
            # fixed membership per window set: a death is handled by aborting
            # the dead peer (ReactiveLink / IpcP2P.abort_peer), not a new epoch
            if getattr(self, "_ipc_key", None) is None:
                self._ipc_key = f"akka/cluster/{int(time.time() * 1e6)}"
            kind = "onesided" if self.transport == "onesided" else "ipc_p2p"
            return {"kind": kind, "store": [self.node.host, int(self._store.port)], "key": self._ipc_key}
        refs = list(self.master.workers.values())
        all_gpu = bool(refs) and all(self._gpu_workers.get(getattr(r, "address", ""), False) for r in refs)
        want_rccl = self.transport == "rccl" or (self.transport == "auto" and all_gpu)
        if not want_rccl:
            return None
        # one unique id per membership: a death or a join starts a new epoch
        # (every member builds a fresh communicator over the new member list)
        members = tuple(sorted(self.master.workers))
        if getattr(self, "_uid_members", None) != members:
            from .._native_loader import load

            self._uid = load().rccl_unique_id()
            self._uid_members = members
        return {"kind": "rccl", "uid": self._uid, "members": list(members)}

    def receive(self, msg: Any) -> None:
        if isinstance(msg, RegisterWorker):
            ref = self.node.ref(msg.address)
            # known before member_up: the join that fills the cluster triggers InitWorkers
            self._gpu_workers[msg.address] = msg.device is not None
            wid = self.master.member_up(ref) if self.master.worker_id(ref) is None else self.master.worker_id(ref)
            if wid is not None:
                self.last_seen[wid] = time.time()
        elif isinstance(msg, Heartbeat):
            self.last_seen[int(msg.srcId)] = time.time()
            if msg.metrics is not None:
                self.node_metrics[int(msg.srcId)] = msg.metrics
        elif isinstance(msg, CompleteAllreduce):
            self.last_seen[int(msg.srcId)] = time.time()
            self.master.receive(msg)
        elif isinstance(msg, WorkerTerminated):
            self.last_seen.pop(int(msg.workerId), None)
            self.master.terminated(int(msg.workerId))
        else:
            self.master.receive(msg)

    def _send_failed(self, address: str, err: BaseException) -> None:
        for wid, ref in list(self.master.workers.items()):
            if getattr(ref, "address", None) == address:
                self.node.mailbox.put(WorkerTerminated(wid))

    def _failure_detector(self) -> None:
        while not self.node.stopped and not self.finished.is_set():
            time.sleep(min(self.heartbeat_interval_s, 0.5))
            now = time.time()
            for wid, t in list(self.last_seen.items()):
                if now - t > self.unreachable_after_s and wid in self.master.workers:
                    log.warning("master: worker %d unreachable for %.1fs -> down", wid, now - t)
                    self.last_seen.pop(wid, None)
                    self.node.mailbox.put(WorkerTerminated(wid))

    def _finished(self) -> None:
        log.info("master: maxRound %d reached", self.master.maxRound)
        for ref in list(self.master.workers.values()):
            ref.tell(Shutdown("maxRound reached"))
        self.finished.set()

    def wait(self, timeout: Optional[float] = None) -> bool:
        return self.finished.wait(timeout)

    def stop(self, join_s: float = 5.0) -> None:
        """Stop the node and wait (bounded) for its threads: a dispatch thread
        still inside native engine code when the interpreter exits would be
        torn down mid-call (pthread_exit unwinding through C++ frames aborts
        the process)."""
        self.node.stop()
        self.node.join(join_s)
        if self._fd is not threading.current_thread():
            self._fd.join(join_s)


def start_master(thresholds: ThresholdConfig, data: DataConfig, workers: WorkerConfig, **kw) -> MasterProcess:
    """AllreduceMaster.startUp(port, thresholds, dataConfig, workerConfig) (M:138-144)."""
    return MasterProcess(thresholds, data, workers, **kw)


# ---------------------------------------------------------------------------
# worker

class WorkerProcess:
    def __init__(self, master_address: str, data_source, data_sink, *, host: str = "127.0.0.1", port: int = 0,
                 device: Any = "cpu", dtype: torch.dtype = torch.float32, heartbeat_interval_s: float = 1.0,
                 transport: str = "auto", metrics_interval_s: float = 0.0):
        self.node = Node(host, port, name="worker")
        dev = torch.device(device) if device not in (None, "cpu") else torch.device("cpu")
        if transport == "auto":
            transport = "stream" if dev.type == "cuda" else "outbox"
        if transport in ("stream", "reactive") and dev.type != "cuda":
            raise ValueError(f"{transport} transport needs a GPU worker")
        if transport == "onesided":
            # threshold rounds over mapped peer windows (GPU) or shared memory
            # (CPU): fast workers never wait for a straggler; master pacing
            # with thAllreduce on top (parallel/onesided_worker.py)
            from .onesided_worker import OneSidedWorker

            self.worker = OneSidedWorker(data_source, data_sink, device=dev, dtype=dtype,
                                         name=f"worker@{self.node.address}")
        else:
            self.worker = AllreduceWorker(data_source, data_sink, device=dev, dtype=dtype, transport=transport,
                                          name=f"worker@{self.node.address}")
        self.stopped = threading.Event()
        self.node.aliases.append(self.worker)
        if hasattr(self.worker, "consume_frames"):
            self.node.frame_consumer = self.worker.consume_frames  # data frames to the native codec
        if transport == "reactive":
            # the dispatcher thread drives the in-flight transfers between messages
            self.node.poller = self._poll
        self.node.start(self)
        self.master = self.node.ref(master_address)
        self.master.tell(RegisterWorker(self.node.address, dev.index if dev.type == "cuda" else None,
                                        socket.gethostname()))
        self.metrics_interval_s = metrics_interval_s
        self._hb = threading.Thread(target=self._heartbeat, args=(heartbeat_interval_s,), daemon=True,
                                    name="worker-hb")
        self._hb.start()

    @property
    def address(self) -> str:
        return self.node.address

    def receive(self, msg: Any) -> None:
        if isinstance(msg, Shutdown):
            log.info("%s: shutdown (%s)", self.worker.name, msg.reason)
            if hasattr(self.worker, "close"):
                self.worker.close()
            self.stopped.set()
            self.node.stop()
            return
        self.worker.receive(msg)

    def _poll(self) -> Optional[bool]:
        core = getattr(self.worker, "_core", None)
        if core is None or not self.worker.initialized or core.in_flight() == 0:
            return None
        return self.worker.poll()

    def _heartbeat(self, interval: float) -> None:
        last_metrics = 0.0
        while not self.stopped.is_set():
            time.sleep(interval)
            if self.worker.initialized and not self.stopped.is_set():
                metrics = None
                now = time.time()
                if self.metrics_interval_s > 0 and now - last_metrics >= self.metrics_interval_s:
                    from ..utils.node_metrics import sample

                    metrics, last_metrics = sample(), now
                try:
                    hb = Heartbeat(self.worker.id, self.worker.round, metrics)
                except AttributeError:
                    return  # the worker was closed under this thread (the job's end)
                self.master.tell(hb)

    def wait(self, timeout: Optional[float] = None) -> bool:
        return self.stopped.wait(timeout)

    def stop(self, join_s: float = 5.0) -> None:
        """Stop and wait (bounded) for the node's and the heartbeat's threads
        (see MasterProcess.stop)."""
        self.stopped.set()
        self.node.stop()
        self.node.join(join_s)
        if self._hb is not threading.current_thread():
            self._hb.join(join_s)


def start_worker(master_address: str, data_size: int, *, checkpoint: int = 50, assert_multiple: int = 0,
                 port: int = 0, device: Any = "cpu", dtype: torch.dtype = torch.float32, printer=print,
                 data_source=None, data_sink=None, **kw) -> WorkerProcess:
    """AllreduceWorker.startUp(port, dataSize, checkpoint, assertMultiple) (W:348-362)."""
    source = data_source or constant_source(data_size, dtype)
    sink = data_sink or ThroughputSink(data_size, checkpoint, assert_multiple, printer=printer)
    return WorkerProcess(master_address, source, sink, port=port, device=device, dtype=dtype, **kw)
