"""Fault injection (the reference has none in code; its tests
hand-craft missing, late, duplicate and out-of-order messages).

* ``FaultyRef`` wraps any actor reference (``tell(msg, sender)``) and drops,
  duplicates or delays the data messages sent through it -- seeded, so a
  failing schedule replays exactly.  Works with every message transport
  (TestKit probe, ``LocalSystem``, TCP ``Node`` refs).
* ``straggler_source`` wraps a data source so one worker is slow to produce
  its input (BASELINE config 4: "an injected sleep in one rank's data source").
* ``env_straggler_delay`` reads ``AKKA_FAULT_RANK`` / ``AKKA_FAULT_DELAY_MS``
  so SPMD jobs (bench, torchrun) can inject a straggler without code changes.
"""
from __future__ import annotations

import os
import random
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional, Tuple, Type

from ..messages import ReduceBlock, ScatterBlock


@dataclass
class FaultStats:
    sent: int = 0
    dropped: int = 0
    duplicated: int = 0
    delayed: int = 0
    log: List[Tuple[str, str]] = field(default_factory=list)  # (action, message type)


class FaultyRef:
    """Actor reference that misbehaves on data messages.

    drop / dup: probabilities per message; delay_s: fixed delay (or a callable
    ``msg -> seconds``) applied on a timer thread, so later messages may
    overtake delayed ones (reordering).  Only ``kinds`` are affected; control
    messages (InitWorkers, StartAllreduce, ...) pass through untouched.
    """

    def __init__(self, ref: Any, *, drop: float = 0.0, dup: float = 0.0,
                 delay_s: float | Callable[[Any], float] = 0.0, seed: int = 0,
                 kinds: Tuple[Type, ...] = (ScatterBlock, ReduceBlock)):
        self.ref = ref
        self.drop = drop
        self.dup = dup
        self.delay_s = delay_s
        self.kinds = kinds
        self.rng = random.Random(seed)
        self.stats = FaultStats()
        self._lock = threading.Lock()

    # the wrapped worker is still "the same actor" for local short-circuit checks
    @property
    def actor(self) -> Any:
        return getattr(self.ref, "actor", self.ref)

    def _deliver(self, msg: Any, sender: Any) -> None:
        self.ref.tell(msg, sender)

    def tell(self, msg: Any, sender: Any = None) -> None:
        if not isinstance(msg, self.kinds):
            self._deliver(msg, sender)
            return
        with self._lock:
            self.stats.sent += 1
            r_drop, r_dup = self.rng.random(), self.rng.random()
            delay = self.delay_s(msg) if callable(self.delay_s) else self.delay_s
            name = type(msg).__name__
            if r_drop < self.drop:
                self.stats.dropped += 1
                self.stats.log.append(("drop", name))
                return
            copies = 2 if r_dup < self.dup else 1
            if copies == 2:
                self.stats.duplicated += 1
                self.stats.log.append(("dup", name))
        for _ in range(copies):
            if delay > 0:
                with self._lock:
                    self.stats.delayed += 1
                t = threading.Timer(delay, self._deliver, args=(msg, sender))
                t.daemon = True
                t.start()
            else:
                self._deliver(msg, sender)

    def __repr__(self) -> str:
        return f"FaultyRef({self.ref!r}, drop={self.drop}, dup={self.dup})"


def straggler_source(source: Callable[[Any], Any], delay_s: float,
                     rounds: Optional[Callable[[int], bool]] = None) -> Callable[[Any], Any]:
    """Data source that sleeps ``delay_s`` before producing (selected) rounds."""

    def slow(req: Any) -> Any:
        if rounds is None or rounds(int(getattr(req, "iteration", 0))):
            time.sleep(delay_s)
        return source(req)

    return slow


def env_straggler_delay(rank: int) -> float:
    """Seconds this rank should sleep before each round (0 if not the faulty rank).

    ``AKKA_FAULT_RANK`` (default: none) and ``AKKA_FAULT_DELAY_MS``.
    """
    want = os.environ.get("AKKA_FAULT_RANK")
    if want is None or int(want) != int(rank):
        return 0.0
    return float(os.environ.get("AKKA_FAULT_DELAY_MS", "0")) / 1e3


def env_phase_stall(rank: int, phase: str) -> None:
    """Hang forever at the start of ``phase`` if ``AKKA_FAULT_STALL_RANK`` names
    this rank and ``AKKA_FAULT_STALL_PHASE`` names the phase: a rank that never
    posts its side of a collective (tests the phase watchdog's failure line).
    ``AKKA_FAULT_STALL_MODE=raise`` raises instead (a rank-local error)."""
    want = os.environ.get("AKKA_FAULT_STALL_RANK")  # a rank, or "all"
    if want is None or (want != "all" and int(want) != int(rank)) or os.environ.get("AKKA_FAULT_STALL_PHASE") != phase:
        return
    if os.environ.get("AKKA_FAULT_STALL_MODE") == "raise":
        raise RuntimeError(f"injected fault on rank {rank} in phase {phase}")
    while True:
        time.sleep(3600)


def env_bad_handoff(rank: int, handoff: str) -> bool:
    """``AKKA_FAULT_BAD_HANDOFF=<mode>`` (e.g. ``lite``): this rank's
    validation rounds of config 4 count one chunk as torn while the lane runs
    in that hand-off mode -- exercises the switch to the fenced hand-off
    without a link that actually reorders (``AKKA_FAULT_BAD_HANDOFF_RANK``
    narrows it to one rank)."""
    want = os.environ.get("AKKA_FAULT_BAD_HANDOFF")
    who = os.environ.get("AKKA_FAULT_BAD_HANDOFF_RANK")
    return want == handoff and (who is None or int(who) == int(rank))


def env_corrupt_round(rank: int, lane: str) -> int:
    """``AKKA_FAULT_CORRUPT_LANE=<lane>``: the index of the round of
    ``ThresholdAllreduce.tune()``'s validation burst in which this rank
    corrupts one element of the lane's output (``AKKA_FAULT_CORRUPT_ROUND``,
    default 7), or -1.  ``AKKA_FAULT_CORRUPT_RANK`` (default 0) picks the
    rank.  Stands in for a data-after-flag reorder on a real link: the
    candidate must be disqualified and its fenced twin chosen."""
    if os.environ.get("AKKA_FAULT_CORRUPT_LANE") != lane:
        return -1
    if int(os.environ.get("AKKA_FAULT_CORRUPT_RANK", "0")) != int(rank):
        return -1
    return int(os.environ.get("AKKA_FAULT_CORRUPT_ROUND", "7"))
