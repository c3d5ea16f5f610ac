"""N-rank simulation of the production (RCCL) schedule on the CPU.

Every rank is a real ``AllreduceWorker`` on the ``stream`` transport; its
device is a deferred host device and its p2p endpoint the native simulator
(``csrc/transport/sim_p2p.cpp``), which implements RCCL's grouped p2p
semantics: rendezvous sends, per-pair in-order matching, whole-group
completion, size checks, and deadlock detection.  So the exact step schedule
that runs over xGMI on MI355X -- group composition, matching order, lag,
counts exchange, stream-ordered arrival -- is validated bit-for-bit here.
"""
from __future__ import annotations

import weakref
from typing import List, Sequence

import torch

from .._native_loader import load as _load
from ..data import AllReduceOutput
from ..messages import InitWorkers
from ..worker import AllreduceWorker
from .collective import _RemoteRank


# Every live simulated cluster (tests/conftest.py checks their race reports
# after each test when AKKA_RACECHECK=1).
LIVE_CLUSTERS: "weakref.WeakSet" = weakref.WeakSet()


class SimCluster:
    def __init__(self, n: int, data_size: int, max_chunk_size: int, *, dtype: torch.dtype = torch.float32,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1, broadcast_lag=2,
                 lane: str = "auto", collectives: bool = False):
        """``collectives``: the simulated communicator also offers RCCL's
        reduce-scatter / all-gather (the exact-round collective lane).  With
        ``AKKA_RACECHECK=1`` in the environment every rank's simulated device
        checks its stream ordering (csrc/engine/racecheck.h) and each worker
        gets a modelled caller stream (``host_stream``)."""
        nat = _load()
        self.n = n
        self.hub = nat.SimHub(n, collectives)
        lags = broadcast_lag if isinstance(broadcast_lag, (list, tuple)) else [broadcast_lag] * n
        self.workers: List[AllreduceWorker] = [
            AllreduceWorker(None, None, device="cpu", dtype=dtype, transport="stream",
                            transport_spec=("sim", self.hub, r), broadcast_lag=lags[r], strict=True, name=f"sim{r}")
            for r in range(n)
        ]
        for r, w in enumerate(self.workers):
            peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
            w.tell(InitWorkers(peers, n, None, r, th_reduce, th_complete, max_lag, data_size, max_chunk_size))
            w.set_lane(lane)
            if w._core.models_streams():  # (the device exists once the worker is initialised)
                w.host_stream = w._core.create_stream()
        LIVE_CLUSTERS.add(self)

    def allreduce(self, inputs: Sequence[torch.Tensor]) -> List[AllReduceOutput]:
        """One round on every rank; returns each rank's output (valid after the simulated run)."""
        assert len(inputs) == self.n
        outs = [w.allreduce(x) for w, x in zip(self.workers, inputs)]
        self.run()
        return outs

    def run(self) -> None:
        _load().sim_run(self.hub, [w._core for w in self.workers])

    def bytes_moved(self) -> int:
        return self.hub.bytes_moved()

    def race_reports(self) -> List[str]:
        """Every rank's stream race reports (AKKA_RACECHECK=1), prefixed by rank."""
        return [f"rank {r}: {m}" for r, w in enumerate(self.workers) for m in w._core.race_reports()]


class ReactiveSimCluster:
    """N ranks on the reactive (straggler-tolerant) transport, on the CPU.

    Same production code as on MI355X -- ReactiveLink with one stream per peer,
    per-pair grouped p2p, event-polled arrivals, staged data plane -- over the
    p2p simulator.  The driver decides which ranks' streams advance and when
    each rank's host polls, so stragglers, frozen ranks and arbitrary stream
    interleavings are reproducible.
    """

    def __init__(self, n: int, data_size: int, max_chunk_size: int, *, dtype: torch.dtype = torch.float32,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1, seed: int = 0):
        import random

        nat = _load()
        self._nat = nat
        self.n = n
        self.hub = nat.SimHub(n)
        self.rng = random.Random(seed)
        self.workers: List[AllreduceWorker] = [
            AllreduceWorker(None, None, device="cpu", dtype=dtype, transport="reactive",
                            transport_spec=("sim", self.hub, r), strict=True, name=f"rsim{r}")
            for r in range(n)
        ]
        for r, w in enumerate(self.workers):
            peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
            w.tell(InitWorkers(peers, n, None, r, th_reduce, th_complete, max_lag, data_size, max_chunk_size))
            if w._core.models_streams():  # AKKA_RACECHECK=1: modelled caller stream
                w.host_stream = w._core.create_stream()
        self.outputs: List[dict] = [dict() for _ in range(n)]
        LIVE_CLUSTERS.add(self)

    def start(self, rank: int, x: torch.Tensor) -> None:
        """Rank ``rank`` starts its next round with contribution ``x``."""
        o = self.workers[rank].allreduce(x)
        if o is not None:
            # completed inside the call: keep it -- the simulated streams may
            # still have ops queued that write its tensors
            self.outputs[rank][o.iteration] = o
        self._collect(rank)

    def _collect(self, rank: int) -> None:
        w = self.workers[rank]
        for r in list(w._outputs):
            self.outputs[rank][r] = w._outputs.pop(r)

    def step(self, active: Sequence[int] = None, shuffle: bool = False) -> bool:
        """Advance the streams of the ``active`` ranks once, then let them poll."""
        active = list(range(self.n)) if active is None else list(active)
        if shuffle:
            self.rng.shuffle(active)
        rot = self.rng.randrange(1 << 16) if shuffle else 0
        moved = bool(self._nat.sim_step(self.hub, [self.workers[r]._core for r in active], rot))
        for r in active:
            moved |= self.workers[r].poll()
            self._collect(r)
        return moved

    def run(self, until, active: Sequence[int] = None, shuffle: bool = False, max_idle: int = 50,
            max_steps: int = 1_000_000) -> None:
        """Step until ``until()`` holds; raise if nothing moves for ``max_idle`` steps."""
        idle = 0
        for _ in range(max_steps):
            if until():
                return
            if self.step(active, shuffle):
                idle = 0
            else:
                idle += 1
                if idle > max_idle:
                    raise RuntimeError("reactive sim: no progress (deadlock) -- "
                                       + "; ".join(f"rank {r}: in_flight={w._core.in_flight()} round={w.round}"
                                                   for r, w in enumerate(self.workers)))
        raise RuntimeError("reactive sim: step budget exhausted")

    def race_reports(self) -> List[str]:
        return [f"rank {r}: {m}" for r, w in enumerate(self.workers) for m in w._core.race_reports()]

    def done(self, rank: int, round_: int) -> bool:
        return round_ in self.outputs[rank]

    def drain(self, active: Sequence[int] = None) -> None:
        """Run until every in-flight transfer of the active ranks finished."""
        ranks = list(range(self.n)) if active is None else list(active)
        self.run(lambda: all(self.workers[r]._core.in_flight() == 0 for r in ranks), active)

    def settle(self, active: Sequence[int] = None) -> None:
        """Run the active ranks' streams until nothing moves (outputs are then readable)."""
        quiet = 0
        while quiet < 3:
            quiet = 0 if self.step(active) else quiet + 1
