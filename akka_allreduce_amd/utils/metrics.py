"""Per-round metrics: round latency, throughput, contributor
counts, forced completions -- as JSON lines.

``MetricsSink`` wraps any data sink; ``worker_summary`` turns the native
engine's counters into a flat dict.
"""
from __future__ import annotations

import json
import time
from typing import Any, Callable, Dict, IO, Optional

from ..data import AllReduceOutput


class MetricsSink:
    """Records one JSON line per completed round, then forwards to ``inner``."""

    def __init__(self, inner: Optional[Callable[[AllReduceOutput], None]] = None, out: Optional[IO[str]] = None,
                 with_counts: bool = False):
        self.inner = inner
        self.out = out
        self.with_counts = with_counts
        self.rows: list[Dict[str, Any]] = []
        self._last = time.perf_counter()

    def __call__(self, r: AllReduceOutput) -> None:
        now = time.perf_counter()
        row: Dict[str, Any] = {"round": r.iteration, "host_dt_ms": round((now - self._last) * 1e3, 4),
                               "bytes": r.data.numel() * r.data.element_size()}
        if self.with_counts:
            c = r.count
            row.update(count_min=int(c.min()), count_max=int(c.max()), count_mean=float(c.float().mean()),
                       missing=int((c == 0).sum()))
        self._last = now
        self.rows.append(row)
        if self.out is not None:
            self.out.write(json.dumps(row) + "\n")
        if self.inner is not None:
            self.inner(r)


def worker_summary(worker) -> Dict[str, Any]:
    st = worker.state()
    d = {"id": st["id"], "round": st["round"], "max_round": st["max_round"]}
    d.update({f"stats_{k}": v for k, v in st["stats"].items()})
    if "link" in st:
        d.update({f"link_{k}": v for k, v in st["link"].items()})
    return d
