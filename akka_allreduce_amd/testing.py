"""TestKit equivalent for driving a single worker by hand.

The reference's ``AllReduceSpec`` (src/test/scala/AllreduceSpec.scala) runs one
real worker and makes every peer *and* the master the TestKit probe
(SPEC:812-818), so a test both plays the other workers and observes every
outgoing message in order.  ``TestProbe`` is that probe: any reference with a
``tell`` method can stand in for a peer or master.  Delivery here is
synchronous, so ``expect_no_msg`` needs no timeout (the reference's
``expectNoMsg`` waits for the default 3 s each time).
"""
from __future__ import annotations

from collections import deque
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch

from .data import AllReduceInput, AllReduceInputRequest, AllReduceOutput
from .messages import ReduceBlock, ScatterBlock


def _as_list(v: Any) -> List[float]:
    if isinstance(v, torch.Tensor):
        return [float(x) for x in v.float().cpu().reshape(-1).tolist()]
    return [float(x) for x in v]


class TestProbe:
    __test__ = False  # not a pytest class

    def __init__(self, name: str = "probe"):
        self.name = name
        self.queue: deque = deque()

    def tell(self, msg: Any, sender: Any = None) -> None:
        self.queue.append(msg)

    # -- expectations ---------------------------------------------------------
    def receive_one(self) -> Any:
        if not self.queue:
            raise AssertionError(f"{self.name}: expected a message, mailbox is empty")
        return self.queue.popleft()

    def expect_msg(self, expected: Any) -> Any:
        m = self.receive_one()
        if m != expected:
            raise AssertionError(f"{self.name}: expected {expected!r}, got {m!r}")
        return m

    def expect_scatter(self, value: Sequence[float], srcId: int, destId: int, chunkId: int, round: int) -> ScatterBlock:
        m = self.receive_one()
        if not isinstance(m, ScatterBlock):
            raise AssertionError(f"{self.name}: expected ScatterBlock, got {m!r}")
        got = (m.srcId, m.destId, m.chunkId, m.round, _as_list(m.value))
        want = (srcId, destId, chunkId, round, [float(x) for x in value])
        if got != want:
            raise AssertionError(f"{self.name}: ScatterBlock mismatch: got {got}, want {want}")
        return m

    def expect_reduce(self, value: Sequence[float], srcId: int, destId: int, chunkId: int, round: int,
                      count: int) -> ReduceBlock:
        m = self.receive_one()
        if not isinstance(m, ReduceBlock):
            raise AssertionError(f"{self.name}: expected ReduceBlock, got {m!r}")
        got = (m.srcId, m.destId, m.chunkId, m.round, m.count, _as_list(m.value))
        want = (srcId, destId, chunkId, round, count, [float(x) for x in value])
        if got != want:
            raise AssertionError(f"{self.name}: ReduceBlock mismatch: got {got}, want {want}")
        return m

    def expect_no_msg(self) -> None:
        if self.queue:
            raise AssertionError(f"{self.name}: expected no message, got {list(self.queue)!r}")

    def fish_for_message(self, pred: Callable[[Any], bool]) -> Any:
        """Skip messages until ``pred`` returns True (raises if it raises)."""
        while True:
            m = self.receive_one()
            if pred(m):
                return m

    def drain(self) -> List[Any]:
        out = list(self.queue)
        self.queue.clear()
        return out


def initialize_workers_as(ref: Any, size: int) -> Dict[int, Any]:
    """Every worker id -> ``ref`` (SPEC:812-818)."""
    return {i: ref for i in range(size)}


def create_custom_data_source(size: int, fn: Callable[[int, int], float]) -> Callable[[AllReduceInputRequest], AllReduceInput]:
    """data[i] = fn(i, iteration) (SPEC:29-35)."""

    def source(req: AllReduceInputRequest) -> AllReduceInput:
        return AllReduceInput(torch.tensor([fn(i, req.iteration) for i in range(size)], dtype=torch.float32))

    return source


def create_basic_data_source(size: int) -> Callable[[AllReduceInputRequest], AllReduceInput]:
    """data[i] = i + iteration (SPEC:23-27)."""
    return create_custom_data_source(size, lambda i, it: float(i + it))


def assertive_data_sink(expected_output: List[List[float]], expected_count: List[List[int]],
                        iterations: List[int], seen: Optional[List[int]] = None) -> Callable[[AllReduceOutput], None]:
    """Sink that checks data and counts of the listed iterations (SPEC:37-44)."""

    def sink(r: AllReduceOutput) -> None:
        assert r.iteration in iterations, f"unexpected iteration {r.iteration}"
        pos = iterations.index(r.iteration)
        assert _as_list(r.data) == [float(x) for x in expected_output[pos]], (
            f"round {r.iteration}: data {_as_list(r.data)} != {expected_output[pos]}")
        got_c = [int(x) for x in r.count.cpu().tolist()]
        assert got_c == list(expected_count[pos]), f"round {r.iteration}: count {got_c} != {expected_count[pos]}"
        if seen is not None:
            seen.append(r.iteration)

    return sink


def collecting_sink(store: List[AllReduceOutput]) -> Callable[[AllReduceOutput], None]:
    def sink(r: AllReduceOutput) -> None:
        store.append(r)

    return sink
