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
                 device: Optional[torch.device] = None, lane: str = "auto"):
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
            w.set_lane(lane)

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


class ReactiveLoopbackCluster:
    """N ranks of the reactive (straggler-tolerant) transport on ONE GPU.

    Each rank: its own HIP streams (one per peer + comm + compute), staged data
    plane, ReactiveLink; the p2p endpoint is the asynchronous per-pair loopback
    (device copies released by stream write-value, never a host rendezvous), so
    a rank whose thread sleeps stalls only its own pairs -- the GPU analogue of
    the CPU simulator's frozen rank.  Needs GPU_MAX_HW_QUEUES >= streams in the
    process (set before the first HIP call; tests/conftest.py does it).
    """

    def __init__(self, n: int, data_size: int, max_chunk_size: int, *, dtype: torch.dtype = torch.float32,
                 th_reduce: float = 1.0, th_complete: float = 1.0, max_lag: int = 1,
                 device: Optional[torch.device] = None):
        self.n = n
        self.hub = _load().PairLoopbackHub(n)
        dev = device or torch.device("cuda", 0)
        self.workers: List[AllreduceWorker] = [
            AllreduceWorker(None, None, device=dev, dtype=dtype, transport="reactive",
                            transport_spec=("loopback_pair", self.hub, r), strict=True, name=f"rlb{r}")
            for r in range(n)
        ]
        for r, w in enumerate(self.workers):
            peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
            w.tell(InitWorkers(peers, n, None, r, th_reduce, th_complete, max_lag, data_size, max_chunk_size))

    def run_rounds(self, inputs: Sequence[Sequence[torch.Tensor]], delays: Optional[Sequence[float]] = None,
                   timeout: float = 45.0) -> List[List[AllReduceOutput]]:
        """Every rank runs len(inputs) rounds back to back (rank r's input of
        round k is inputs[k][r]); rank r first sleeps delays[r] seconds.
        Returns outs[rank][round] (each made valid on the caller's stream)."""
        import time

        outs: List[List[Optional[AllReduceOutput]]] = [[None] * len(inputs) for _ in range(self.n)]
        errs: List[BaseException] = []

        def run(r: int) -> None:
            try:
                if delays and delays[r]:
                    time.sleep(delays[r])
                w = self.workers[r]
                w.reactive_timeout = timeout
                for k, xs in enumerate(inputs):
                    outs[r][k] = w.allreduce(xs[r])
                torch.cuda.current_stream().synchronize()
            except BaseException as e:  # pragma: no cover - surfaced below
                errs.append(e)

        ts = [threading.Thread(target=run, args=(r,)) for r in range(self.n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            self.hub.release_all()  # never leave streams parked on a dead schedule
            raise errs[0]
        return outs  # type: ignore[return-value]

    def close(self) -> None:
        """Drain, then free every rank's streams and buffers (deterministically:
        a hipFree from a later garbage collection would synchronize the device
        while another cluster's streams wait for their peers)."""
        import gc

        try:
            self.drain()
        finally:
            for w in self.workers:
                w.close()
            self.workers = []
            self.hub = None
            gc.collect()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def drain(self, timeout: float = 60.0) -> None:
        """Poll every rank until all in-flight transfers finished."""
        import time

        t0 = time.monotonic()
        while any(w._core.in_flight() for w in self.workers):
            for w in self.workers:
                w.poll()
            if time.monotonic() - t0 > timeout:
                self.hub.release_all()
                raise TimeoutError("reactive loopback: transfers still in flight")
