"""Executable specification of one worker, in plain Python.

This is the reference worker's state machine (AllreduceWorker.scala:7-301
with ScatteredDataBuffer / ReducedDataBuffer, SURVEY §2.6 rules 1-8) written
as directly as possible, with this framework's deliberate quirk fixes
(SURVEY §5.3): thresholds fire once at ``>=`` over distinct sources, exact
integer partitioning with empty trailing blocks, no catch-up double-complete,
scatter/broadcast loop over all N ids.  ``tests/test_model_diff.py`` drives
it and the native engine with the same random message sequences and compares
every emitted message and every sink output.
"""
from __future__ import annotations

import numpy as np


def float_threshold(th: float, n: int) -> int:
    return int(np.float32(th) * np.float32(n))


class Geometry:
    def __init__(self, S: int, N: int, C: int):
        self.S, self.N, self.C = S, N, C
        self.step = (S + N - 1) // N

    def block_start(self, j):
        return min(j * self.step, self.S)

    def block_end(self, j):
        return self.S if j >= self.N - 1 else min((j + 1) * self.step, self.S)

    def block_len(self, j):
        return self.block_end(j) - self.block_start(j)

    def num_chunks(self, j):
        return (self.block_len(j) + self.C - 1) // self.C

    def chunk_len(self, j, k):
        return min(self.C, self.block_len(j) - k * self.C)

    def chunk_offset(self, j, k):
        return self.block_start(j) + k * self.C

    def total_chunks(self):
        return sum(self.num_chunks(j) for j in range(self.N))


class ModelWorker:
    """Emits ('scatter', src, dest, chunk, round, values), ('reduce', src, dest,
    chunk, round, count, values) and ('complete', src, round) into ``out``;
    sink outputs (round, data, counts) into ``sink``."""

    def __init__(self, source, *, self_local: bool = False):
        self.source = source
        self.self_local = self_local
        self.out = []
        self.sink = []

    def init(self, id_, N, th_reduce, th_complete, max_lag, S, C, peers=None):
        self.peers = set(range(N)) if peers is None else set(peers)
        self.id, self.N, self.max_lag = id_, N, max_lag
        self.g = Geometry(S, N, C)
        self.kme = self.g.num_chunks(id_)
        self.min_scatter = min(max(float_threshold(th_reduce, N), 1), N)
        total = self.g.total_chunks()
        self.min_reduced = min(max(float_threshold(th_complete, total), 1), max(total, 1))
        self.round, self.max_round, self.max_scattered = 0, -1, -1
        self.completed = set()
        self.rows = {}  # round -> state
        self.inputs = {}

    def reinit(self, peers):
        self.peers = set(peers)  # re-init only replaces the peer map (W:87-89)

    def terminated(self, id_):
        self.peers.discard(id_)

    # ---- per-round state (a ring row of the reference) ------------------------
    def row(self, r):
        if r not in self.rows:
            self.rows[r] = {"slots": {}, "mask": {}, "reduced": set(), "landed": {}, "done": False}
        return self.rows[r]

    # ---- handlers -----------------------------------------------------------------
    def start(self, r):
        self.max_round = max(self.max_round, r)
        while self.round < self.max_round - self.max_lag:  # catch-up (W:100-106)
            r0 = self.round
            for k in range(self.kme):
                if self.round != r0:
                    break
                if k not in self.row(r0)["reduced"]:
                    self.reduce_and_broadcast(r0, k)
            if r0 not in self.completed:
                self.complete(r0)
        while self.max_scattered < self.max_round:
            nxt = self.max_scattered + 1
            self.inputs[nxt] = [float(v) for v in self.source(nxt)]
            self.scatter(nxt)
            self.max_scattered = nxt
        self.completed = {c for c in self.completed if c >= self.round}

    def scatter(self, r):
        data = self.inputs[r]
        for i in range(self.N):
            idx = (i + self.id) % self.N
            if idx not in self.peers:
                continue
            for k in range(self.g.num_chunks(idx)):
                o = self.g.chunk_offset(idx, k)
                val = data[o:o + self.g.chunk_len(idx, k)]
                if idx == self.id and self.self_local:
                    self.on_scatter(self.id, idx, k, r, val)
                else:
                    self.out.append(("scatter", self.id, idx, k, r, val))

    def on_scatter(self, src, dest, chunk, r, val):
        if r < self.round or r in self.completed:
            return
        if r > self.max_round:
            self.start(r)
            return self.on_scatter(src, dest, chunk, r, val)
        rw = self.row(r)
        rw["slots"][(src, chunk)] = list(val)
        rw["mask"].setdefault(chunk, set()).add(src)
        if chunk not in rw["reduced"] and len(rw["mask"][chunk]) >= self.min_scatter:
            self.reduce_and_broadcast(r, chunk)

    def reduce_and_broadcast(self, r, chunk):
        rw = self.row(r)
        srcs = sorted(rw["mask"].get(chunk, ()))
        n = self.g.chunk_len(self.id, chunk)
        acc = np.zeros(n, dtype=np.float32)
        for s in srcs:
            acc += np.asarray(rw["slots"][(s, chunk)], dtype=np.float32)
        val = [float(v) for v in acc]
        rw["reduced"].add(chunk)
        # Zero-copy data plane: my reduced chunk is written straight into the
        # output at its final offset.  A ReduceBlock(src=me) that landed there
        # before my own reduce keeps its count but not its values.  Only a
        # harness can produce that order (self mapped to a probe, SPEC-style);
        # the reference would keep the external copy (RB:21-24).
        if (self.id, chunk) in rw["landed"]:
            rw["landed"][(self.id, chunk)] = (rw["landed"][(self.id, chunk)][0], val)
        for i in range(self.N):
            idx = (i + self.id) % self.N
            if idx not in self.peers:
                continue
            if idx == self.id and self.self_local:
                self.on_reduce(self.id, idx, chunk, r, len(srcs), val)
            else:
                self.out.append(("reduce", self.id, idx, chunk, r, len(srcs), val))

    def on_reduce(self, src, dest, chunk, r, count, val):
        if r < self.round or r in self.completed:
            return
        if r > self.max_round:
            self.start(r)
            return self.on_reduce(src, dest, chunk, r, count, val)
        rw = self.row(r)
        rw["landed"][(src, chunk)] = (count, list(val))
        if not rw["done"] and len(rw["landed"]) >= self.min_reduced:
            self.complete(r)

    def complete(self, r):
        rw = self.row(r)
        rw["done"] = True
        data = [0.0] * self.g.S
        counts = [0] * self.g.S
        for (j, k), (c, val) in rw["landed"].items():
            o = self.g.chunk_offset(j, k)
            data[o:o + len(val)] = val
            counts[o:o + len(val)] = [c] * len(val)
        self.sink.append((r, data, counts))
        self.out.append(("complete", self.id, r))
        self.completed.add(r)
        if self.round == r:
            while self.round in self.completed:
                self.round += 1
        del self.rows[r]
