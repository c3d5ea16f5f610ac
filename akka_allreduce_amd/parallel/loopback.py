"""N ranks on ONE GPU in one process (test harness for the GPU data path).

Each rank is a full ``AllreduceWorker`` on the scheduled transport with its
own HIP streams, data plane and StreamLink; only the p2p endpoint differs
from production (device copies + host rendezvous instead of RCCL, which needs
one GPU per rank).  Each rank runs in its own host thread, like one process
per GPU.  Used by the GPU tests to check the real stream/event ordering at
N = 2..8 on a single MI355X.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence

import torch

from .._native_loader import load as _load
from ..data import AllReduceOutput
from ..messages import InitWorkers
from ..worker import AllreduceWorker
from .collective import _RemoteRank


class LoopbackCluster:
    def __init__(self, n: int, data_size: int, max_chunk_size: int, *, dtype: torch.dtype = torch.float32,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1, broadcast_lag: int = 2,
                 device: Optional[torch.device] = None):
        self.n = n
        self.hub = _load().LoopbackHub(n)
        dev = device or torch.device("cuda", 0)
        self.workers: List[AllreduceWorker] = [
            AllreduceWorker(None, None, device=dev, dtype=dtype, transport="stream",
                            transport_spec=("loopback", self.hub, r), broadcast_lag=broadcast_lag, strict=True,
                            name=f"lb{r}")
            for r in range(n)
        ]
        for r, w in enumerate(self.workers):
            peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
            w.tell(InitWorkers(peers, n, None, r, th_reduce, th_complete, max_lag, data_size, max_chunk_size))

    def allreduce(self, inputs: Sequence[torch.Tensor], async_op: bool = False) -> List[AllReduceOutput]:
        assert len(inputs) == self.n
        outs: List[Optional[AllReduceOutput]] = [None] * self.n
        errs: List[BaseException] = []

        def run(r: int) -> None:
            try:
                outs[r] = self.workers[r].allreduce(inputs[r], async_op=async_op)
            except BaseException as e:  # pragma: no cover - surfaced below
                errs.append(e)

        ts = [threading.Thread(target=run, args=(r,)) for r in range(self.n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return outs  # type: ignore[return-value]

    def bytes_moved(self) -> int:
        return self.hub.bytes_moved()
