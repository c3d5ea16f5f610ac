"""AllreduceMaster: membership and round pacing (reference ``AllreduceMaster.scala:12-144``).

Transport-agnostic: workers are references with ``tell(msg)`` (in-process
workers, the TestKit probe, or TCP proxies from ``parallel.cluster``).

Reference behaviour kept:
  * workers get ids in join order; once ``totalWorkers`` have joined, every
    worker receives ``InitWorkers`` and round 0 starts (M:36-44, M:76-81);
  * ``CompleteAllreduce`` for the current round is counted; when
    ``numComplete >= totalWorkers * thAllreduce`` (float32) and
    ``round < maxRound``, the next round starts (M:54-63);
  * completions of other rounds are ignored.

Reference gaps fixed:
  * a dead worker is removed AND the pacing threshold uses the live count, so
    ``thAllreduce = 1`` no longer stalls forever after a death;
  * ids are the smallest free id in ``[0, totalWorkers)`` (the reference's
    ``workers.size`` collides after a removal);
  * surviving workers are told about the death (``WorkerTerminated``); on a
    device (RCCL) data plane they also get a re-``InitWorkers`` carrying a new
    unique id and the survivor list, from which they build a new communicator
    (a membership epoch); and a
    worker joining after the start takes a free id, gets ``InitWorkers`` and the
    current ``StartAllreduce`` (it catches up through the worker's catch-up
    path); the survivors get a re-``InitWorkers`` with the new peer map.
"""
from __future__ import annotations

import logging
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from .config import DataConfig, ThresholdConfig, WorkerConfig
from .messages import CompleteAllreduce, InitWorkers, RegisterWorker, StartAllreduce, WorkerTerminated

log = logging.getLogger("akka_allreduce_amd.master")


class AllreduceMaster:
    def __init__(
        self,
        totalWorkers: int,
        thAllreduce: float,
        thReduce: float,
        thComplete: float,
        maxLag: int,
        dataSize: int,
        maxRound: int,
        maxChunkSize: int,
        *,
        on_round_start: Optional[Callable[[int], None]] = None,
        on_finished: Optional[Callable[[], None]] = None,
        transport_info: Optional[Callable[[], Dict[str, Any]]] = None,
        min_workers: Optional[int] = None,
    ):
        self.totalWorkers = int(totalWorkers)
        # round 0 starts once this many workers joined (the reference waits
        # for all, M:39); fewer starts with a partial peer map and the rest
        # join later (T4/T5, SPEC:141-170: re-InitWorkers with the new map)
        self.min_workers = self.totalWorkers if min_workers is None else max(1, min(int(min_workers),
                                                                                     self.totalWorkers))
        self.thAllreduce = float(thAllreduce)
        self.thReduce = float(thReduce)
        self.thComplete = float(thComplete)
        self.maxLag = int(maxLag)
        self.dataSize = int(dataSize)
        self.maxRound = int(maxRound)
        self.maxChunkSize = int(maxChunkSize)
        self.workers: Dict[int, Any] = {}
        self.round = -1
        self.numComplete = 0
        self.completed_by: Dict[int, List[int]] = {}
        self.on_round_start = on_round_start
        self.on_finished = on_finished
        self.transport_info = transport_info
        self.finished = False

    # ---- config-object constructor (AllreduceMaster.startUp, M:138-144) ------
    @classmethod
    def from_configs(cls, thresholds: ThresholdConfig, data: DataConfig, workers: WorkerConfig, **kw) -> "AllreduceMaster":
        return cls(workers.totalSize, thresholds.thAllreduce, thresholds.thReduce, thresholds.thComplete,
                   workers.maxLag, data.dataSize, data.maxRound, data.maxChunkSize, **kw)

    @staticmethod
    def startUp(port: int, thresholds: ThresholdConfig, dataConfig: DataConfig, workerConfig: WorkerConfig, **kw):
        """Reference entry point ``AllreduceMaster.startUp(port, thresholds,
        dataConfig, workerConfig)`` (M:138-144): a master process listening on
        ``port`` (TCP control plane).  Returns the running ``MasterProcess``."""
        from .parallel.cluster import start_master

        return start_master(thresholds, dataConfig, workerConfig, port=int(port), **kw)

    # ---- actor API -------------------------------------------------------------
    def tell(self, msg: Any, sender: Any = None) -> None:
        self.receive(msg, sender)

    def receive(self, msg: Any, sender: Any = None) -> None:
        if isinstance(msg, CompleteAllreduce):
            self._on_complete(msg)
        elif isinstance(msg, RegisterWorker):
            if sender is None:
                raise ValueError("RegisterWorker needs the worker reference as sender")
            self.member_up(sender)
        elif isinstance(msg, WorkerTerminated):
            self.terminated(int(msg.workerId))
        else:
            raise TypeError(f"master: unhandled message {msg!r}")

    # ---- membership --------------------------------------------------------------
    def _free_id(self) -> Optional[int]:
        for i in range(self.totalWorkers):
            if i not in self.workers:
                return i
        return None

    def member_up(self, ref: Any) -> Optional[int]:
        """A worker joined (MemberUp + register, M:36-44, M:66-74).  Returns its id."""
        for i, r in self.workers.items():
            if r is ref:
                return i
        new_id = self._free_id()
        if new_id is None:
            log.warning("master: cluster full (%d workers), ignoring join", self.totalWorkers)
            return None
        self.workers[new_id] = ref
        log.info("master: worker %d joined (%d/%d)", new_id, len(self.workers), self.totalWorkers)
        if self.round == -1:
            if len(self.workers) >= self.min_workers:
                self._init_workers(list(self.workers))
                self.round = 0
                self._start_allreduce()
        else:
            # elastic re-join into a vacated id: init it, refresh everyone's peer map
            self._init_workers(list(self.workers))
            ref.tell(StartAllreduce(self.round))
        return new_id

    def terminated(self, worker_id: int) -> None:
        """Worker death (Terminated, M:46-52) -- also told to the survivors."""
        if self.workers.pop(worker_id, None) is None:
            return
        log.warning("master: worker %d terminated, %d alive", worker_id, len(self.workers))
        for ref in list(self.workers.values()):
            ref.tell(WorkerTerminated(worker_id))
        if self.round >= 0 and self.transport_info is not None and self.workers:
            # device data plane: the survivors build a new communicator over
            # themselves (new unique id, members = survivors) -- a worker
            # cannot leave an RCCL communicator it shares with a dead rank
            self._init_workers(list(self.workers))
        if self.round >= 0:
            self._maybe_advance()

    def worker_id(self, ref: Any) -> Optional[int]:
        for i, r in self.workers.items():
            if r is ref:
                return i
        return None

    # ---- rounds --------------------------------------------------------------------
    def _init_workers(self, ids: List[int]) -> None:
        extra = self.transport_info() if self.transport_info else None
        if extra is not None:
            extra = dict(extra)
            extra.setdefault("members", sorted(self.workers))
        for idx in ids:
            msg = InitWorkers(dict(self.workers), self.totalWorkers, self, idx, self.thReduce, self.thComplete,
                              self.maxLag, self.dataSize, self.maxChunkSize)
            if extra is not None:
                msg.transport = extra  # type: ignore[attr-defined]
            self.workers[idx].tell(msg)

    def _start_allreduce(self) -> None:
        log.info("master: start allreduce round %d", self.round)
        self.numComplete = 0
        if self.on_round_start:
            self.on_round_start(self.round)
        for ref in list(self.workers.values()):
            ref.tell(StartAllreduce(self.round))

    def _threshold(self) -> float:
        alive = min(len(self.workers), self.totalWorkers)
        return float(np.float32(alive) * np.float32(self.thAllreduce))

    def _maybe_advance(self) -> None:
        if self.numComplete >= self._threshold() and self.round < self.maxRound:
            log.info("master: %d (of %d) workers completed round %d", self.numComplete, len(self.workers), self.round)
            self.round += 1
            self._start_allreduce()
        elif self.numComplete >= self._threshold() and self.round >= self.maxRound and not self.finished:
            self.finished = True
            if self.on_finished:
                self.on_finished()

    def _on_complete(self, c: CompleteAllreduce) -> None:
        self.completed_by.setdefault(int(c.round), []).append(int(c.srcId))
        if int(c.round) == self.round:
            self.numComplete += 1
            self._maybe_advance()
