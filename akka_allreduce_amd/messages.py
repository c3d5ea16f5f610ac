"""Wire protocol: the reference's case classes as Python dataclasses.

Field names and order are kept identical to
``src/main/scala/sample/cluster/allreduce/AllreduceMessage.scala:7-21`` so code
written against the reference's message API reads the same.  ``value`` is a
1-D tensor (the reference's ``Array[Float]``); any sequence or numpy array is
accepted on input and converted by the receiving worker.

Messages that exist only in this framework (membership/liveness, which the
reference delegates to Akka Cluster gossip) are below the
reference set.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class InitWorkers:
    """Master -> worker: membership + thresholds (MSG:7-17).

    ``workers`` maps worker id -> actor reference (anything with ``tell(msg)``;
    the worker recognises itself and short-circuits those messages, W:228).
    """

    workers: Dict[int, Any]
    workerNum: int
    master: Any
    destId: int
    thReduce: float
    thComplete: float
    maxLag: int
    dataSize: int
    maxChunkSize: int


@dataclass
class StartAllreduce:
    """Master -> worker: round ``round`` may start (MSG:18)."""

    round: int


@dataclass
class ScatterBlock:
    """Phase 1 chunk: ``srcId``'s copy of chunk ``chunkId`` of ``destId``'s block (MSG:19)."""

    value: Any
    srcId: int
    destId: int
    chunkId: int
    round: int


@dataclass
class ReduceBlock:
    """Phase 2 chunk: reduced chunk ``chunkId`` of ``srcId``'s block, ``count`` contributors (MSG:20)."""

    value: Any
    srcId: int
    destId: int
    chunkId: int
    round: int
    count: int


@dataclass
class CompleteAllreduce:
    """Worker -> master: ``srcId`` finished round ``round`` (MSG:21)."""

    srcId: int
    round: int


# ---------------------------------------------------------------------------
# Membership / liveness (Akka Cluster MemberUp / Terminated in the reference)


@dataclass
class RegisterWorker:
    """Worker -> master: join request (replaces MemberUp + resolveOne, M:36-44, M:66-74)."""

    address: str = ""
    device: Optional[int] = None
    hostname: str = ""
    meta: Dict[str, Any] = field(default_factory=dict)


@dataclass
class WorkerTerminated:
    """Master -> workers: ``workerId`` is gone (the reference's Terminated, M:46-52 / W:141-146)."""

    workerId: int


@dataclass
class Heartbeat:
    srcId: int
    round: int
    metrics: Optional[Dict[str, Any]] = None  # node metrics sample (utils/node_metrics.py), when enabled


@dataclass
class Shutdown:
    reason: str = ""


def is_data_message(msg: Any) -> bool:
    return isinstance(msg, (ScatterBlock, ReduceBlock))
