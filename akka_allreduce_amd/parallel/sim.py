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

from typing import List, Sequence

import torch

from .._native_loader import load as _load
from ..data import AllReduceOutput
from ..messages import InitWorkers
from ..worker import AllreduceWorker
from .collective import _RemoteRank


class SimCluster:
    def __init__(self, n: int, data_size: int, max_chunk_size: int, *, dtype: torch.dtype = torch.float32,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1, broadcast_lag=2):
        nat = _load()
        self.n = n
        self.hub = nat.SimHub(n)
        lags = broadcast_lag if isinstance(broadcast_lag, (list, tuple)) else [broadcast_lag] * n
        self.workers: List[AllreduceWorker] = [
            AllreduceWorker(None, None, device="cpu", dtype=dtype, transport="stream",
                            transport_spec=("sim", self.hub, r), broadcast_lag=lags[r], strict=True, name=f"sim{r}")
            for r in range(n)
        ]
        for r, w in enumerate(self.workers):
            peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
            w.tell(InitWorkers(peers, n, None, r, th_reduce, th_complete, max_lag, data_size, max_chunk_size))

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
