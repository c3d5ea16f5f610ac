"""The one-sided threshold lane replaying the reference spec's arrival orders.

``AllreduceSpec.scala`` drives ONE real worker and plays every peer (and the
master) with the TestKit probe (SPEC:812-818): it injects ScatterBlock /
ReduceBlock messages in a chosen order and asserts every message the worker
emits.  Here the worker is rank 0's ``OneSidedLane`` on the CPU backend
(csrc/transport/onesided.h: the GPU kernels' protocol functions on shared
memory), stepped with ``begin`` / ``progress``; its pushes are HELD in an
outbox, which the test reads as the probe reads the worker's messages; the
peers are the other ranks' lanes, whose pushes the test injects with
arbitrary bytes through the same gates (``inject``).  Deterministic: nothing
moves unless the test moves it.

Semantics shared with the reference and asserted here: reduce at
floor(thReduce*N) copies over exactly the landed set with count = copies
(SB:9-13, SB:20-32), complete at floor(thComplete*total) reduced chunks with
missing chunks 0 / count 0 (RB:13-17, RB:26-53, RB:60-66), outdated messages
dropped (W:155-156, W:172-173), catch-up at maxLag (W:100-106).

Where the lane differs by design (docs/DESIGN.md, one-sided lane):
  * a rank's own scatter copy is always present (self-delivery, W:228-232);
    the spec's probe sometimes withholds it, so where a spec case relies on
    that the peer copy withheld here is another one, and the values are the
    ones this cluster really sums;
  * a rank serves one round per call, in order; messages of later rounds
    land in their ring rows and are used when that round is served (a chunk
    decided after more copies landed uses all of them: count = copies);
  * a source that already announced a later round is past this one: its
    missing copies end the wait at once (liveness) instead of at maxLag;
  * rounds skipped by catch-up are not re-scattered.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from akka_allreduce_amd._native_loader import load
from model_worker import Geometry


class SpecHarness:
    """Rank ``me`` is the worker under test; the test plays every other rank."""

    def __init__(self, N, S, C, th_reduce, th_complete, max_lag, me=0, rows=0, members=None):
        nat = load()
        self.N, self.S, self.C, self.me = N, S, C, me
        self.g = Geometry(S, N, C)
        self.kmax = max(1, max(self.g.num_chunks(j) for j in range(N)))
        # one part per chunk: a message of the spec is one (chunk, part) push
        self.lanes = [nat.OneSidedLane(-1, S, N, C, r, "float32", th_reduce=th_reduce, th_complete=th_complete,
                                       max_lag=max_lag, rows=rows, part_bytes=1 << 40, timeout_ms=3_600_000)
                      for r in range(N)]
        hs = [ln.handle() for ln in self.lanes]
        self.handles = hs
        for r, ln in enumerate(self.lanes):
            # the worker under test may start with a partial peer map (T4):
            # absent ranks get no window mapping (an empty handle) until admit()
            if r == me and members is not None:
                ln.open([h if q in members or q == me else b"" for q, h in enumerate(hs)])
            else:
                ln.open(hs)
        if members is None:
            for ln in self.lanes:
                ln.unlink()
        self.w = self.lanes[me]
        self.w.set_hold(True)
        self.starts: list = []   # queued calls (input data), served in order
        self.cur = None
        self.outputs: list = []  # (round, data, per-element counts, reason)
        self.sent: list = []     # the worker's pushes, in emission order

    # ---- the worker ---------------------------------------------------------------
    def start(self, data):
        """The worker's next call (StartAllreduce from the master, M:83-89)."""
        self.starts.append([float(v) for v in data])
        self.pump()

    def pump(self):
        while True:
            if self.cur is None and self.starts:
                x = torch.tensor(self.starts.pop(0), dtype=torch.float32)
                out = torch.full((self.S,), float("nan"))
                counts = torch.full((self.N, self.kmax), -1, dtype=torch.int32)
                call = self.w.begin(x.data_ptr(), out.data_ptr(), counts.data_ptr(), self.kmax)
                self.cur = (x, out, counts, call)
            if self.cur is None:
                self._collect()
                return
            done = self.w.progress()
            self._collect()
            if not done:
                return
            x, out, counts, call = self.cur
            st = self.w.status(call)
            per_el = [0] * self.S
            for j in range(self.N):
                for k in range(self.g.num_chunks(j)):
                    o = self.g.chunk_offset(j, k)
                    for e in range(o, o + self.g.chunk_len(j, k)):
                        per_el[e] = int(counts[j, k])
            self.outputs.append((st["round"], [float(v) for v in out.tolist()], per_el, st["reason"]))
            self.cur = None

    def _collect(self):
        ob = self.w.outbox()
        for i, m in enumerate(ob):
            vals = np.frombuffer(self.w.outbox_bytes(i), dtype=np.float32).tolist()
            self.sent.append((m["phase"], m["dst"], m["chunk"], m["round"], m["count"], vals))
        for _ in ob:
            self.w.drop(0)  # the probe received it

    def take_sent(self, phase=None):
        s = [m for m in self.sent if phase is None or m[0] == phase]
        self.sent = [m for m in self.sent if not (phase is None or m[0] == phase)]
        return s

    def admit(self, q):
        """Re-InitWorkers with a larger peer map (W:87-89): the worker maps
        rank q's window between rounds."""
        self.w.add_peer(q, self.handles[q])

    # ---- the peers ------------------------------------------------------------------
    def scatter(self, src, k, r, vals):
        self.lanes[src].inject(0, self.me, k, 0, r, 0, np.asarray(vals, dtype=np.float32).tobytes())
        self.pump()

    def reduce(self, src, k, r, count, vals):
        self.lanes[src].inject(1, self.me, k, 0, r, count, np.asarray(vals, dtype=np.float32).tobytes())
        self.pump()

    def stats(self, rank=None):
        return self.lanes[self.me if rank is None else rank].stats()


def basic(size, it):
    """createBasicDataSource (SPEC:23-27): data[i] = i + iteration."""
    return [float(i + it) for i in range(size)]


def reduces(h, r=None):
    """The worker's ReduceBlocks as (dest, chunk, round, count, values)."""
    return [m[1:] for m in h.take_sent("gather") if r is None or m[3] == r]


def test_t1_sum_up_all_correct_data():
    """SPEC:57-95 (N=2, S=3, C=2, thresholds 1, maxLag 5, worker 1 -- the
    one case where the spec maps the worker's own id to the real worker, so
    its self-delivery runs, W:228-232): two rounds of generator idx + iter.
    Worker 1 owns [2, 3): it scatters block 0 to rank 0, reduces its own
    element from both copies (count 2) and completes each round with 2 x
    input and counts [2, 2, 2] (the spec's assertiveDataSink)."""
    h = SpecHarness(2, 3, 2, 1.0, 1.0, 5, me=1)
    for it in (0, 1):
        x = basic(3, it)
        h.start(x)
        assert [(m[1], m[2], m[3], m[5]) for m in h.take_sent("scatter")] == [(0, 0, it, x[0:2])]
        h.scatter(0, 0, it, [x[2]])  # rank 0's copy of my element (same generator)
        assert reduces(h) == [(0, 0, it, 2, [2 * x[2]])]
        h.reduce(0, 0, it, 2, [2 * x[0], 2 * x[1]])
        assert h.outputs[-1] == (it, [2 * v for v in x], [2, 2, 2], "threshold")
    assert len(h.outputs) == 2


def _t2_early_reduce_of_a_future_round():
    h = SpecHarness(4, 8, 2, 1.0, 0.8, 5)
    h.start(basic(8, 0))
    for s, v in ((1, [11.0, 10.0]), (2, [10.0, 20.0]), (3, [9.0, 10.0])):
        h.reduce(s, 0, 3, 4, v)
    for i in (1, 2, 3):
        h.start(basic(8, i))
    return h


def test_t3_no_longer_act_on_completed_scatter():
    """SPEC:133-138: after round 3 completed (T2's ReduceBlocks), the
    ScatterBlocks of that round from every peer change nothing: no message,
    no output (expectNoMsg); the senders count them as outdated."""
    h = _t2_early_reduce_of_a_future_round()
    assert [o[0] for o in h.outputs] == [0, 1, 2, 3]
    h.take_sent()
    for s in (1, 2, 3):
        h.scatter(s, 0, 3, [2.0 * s, 2.0 * s])
    assert h.take_sent() == [] and len(h.outputs) == 4
    assert sum(h.stats(s)["scatter_outdated"] for s in (1, 2, 3)) == 3


def test_t6_single_round_allreduce():
    """SPEC:175-213 (N=4, S=8, C=2, thR 1, thC 0.75 -> 3): the worker's
    scatters go out in the exact rotated order, self first (delivered in
    place, W:228-232), then ranks 1, 2, 3 with [2i, 2i+1]; the reduce waits
    for all four copies (count 4) and goes to ranks 1, 2, 3 in that order;
    the round completes at the third reduced chunk (own + 2), the fourth is
    outdated.  (The spec's probe plays the worker's own copy as [0, 0]; here
    the worker's real input [0, 1] is summed: [12, 13].)"""
    h = SpecHarness(4, 8, 2, 1.0, 0.75, 5)
    h.start(basic(8, 0))
    assert [(m[1], m[2], m[3], m[5]) for m in h.take_sent("scatter")] == \
        [(i, 0, 0, [2.0 * i, 2.0 * i + 1]) for i in (1, 2, 3)]
    for i in (1, 2):
        h.scatter(i, 0, 0, [2.0 * i, 2.0 * i])
        assert reduces(h) == []
    h.scatter(3, 0, 0, [6.0, 6.0])
    assert reduces(h) == [(d, 0, 0, 4, [12.0, 13.0]) for d in (1, 2, 3)]
    h.reduce(1, 0, 0, 4, [11.0, 10.0])
    assert h.outputs == []
    h.reduce(2, 0, 0, 4, [10.0, 20.0])
    assert h.outputs == [(0, [12.0, 13.0, 11.0, 10.0, 10.0, 20.0, 0.0, 0.0], [4, 4, 4, 4, 4, 4, 0, 0], "threshold")]
    h.reduce(3, 0, 0, 4, [9.0, 10.0])
    assert len(h.outputs) == 1 and h.stats(3)["gather_outdated"] == 1


def test_t7_uneven_size_sending_to_self_first():
    """SPEC:215-238 (N=2, S=3, C=1, thresholds 1, maxLag 1, worker 1):
    blocks [0, 2) and [2, 3); worker 1 delivers its own element to itself
    first (in place), then chunks 0 and 1 of block 0 to rank 0, in order."""
    h = SpecHarness(2, 3, 1, 1.0, 1.0, 1, me=1)
    h.start(basic(3, 0))
    assert [(m[1], m[2], m[3], m[5]) for m in h.take_sent("scatter")] == [(0, 0, 0, [0.0]), (0, 1, 0, [1.0])]
    assert reduces(h) == [] and h.outputs == []  # its own element waits for rank 0's copy


def per_dest(msgs):
    """Messages grouped by destination, each in emission order: the order the
    reference's per-pair FIFO makes observable (W:213-237 sends every chunk to
    a peer in ascending order; across peers -- different links -- the lane's
    interleaving is its own)."""
    out: dict = {}
    for m in msgs:
        out.setdefault(m[1], []).append(m)
    return out


def test_t18_rounds_complete_in_order_using_early_copies():
    """SPEC:664-734 (N=3, S=9, C=2 -> chunks of 2 and 1, thR 0.75 -> 2, thC
    0.75 -> 4 of 6), the lane's documented divergence pinned.  The reference
    scatters round 1 as soon as it is started and completes round 1 BEFORE
    round 0 (out-of-order completion, W:277-284).  The lane serves one round
    per call, in order, and a peer's round-r pushes all precede its round-r+1
    pushes (its call for r+1 starts after its call for r ended), so the
    spec's exact interleaving cannot occur; its point -- a fast peer's next
    round overtaking a slow one's current round -- does: rank 1 runs ahead
    into round 1 while rank 2 still owes round 0.  Rank 1's round-1 copies
    and reduced chunks land early in round 1's ring row; rounds reach the
    sink as 0, then 1; round 1 -- served the moment round 0 completes --
    reduces over the early copies and completes at once from the chunks that
    had landed."""
    h = SpecHarness(3, 9, 2, 0.75, 0.75, 5)
    h.start(basic(9, 0))
    sc = per_dest(h.take_sent("scatter"))
    assert {d: [(m[2], m[3], m[5]) for m in v] for d, v in sc.items()} == \
        {1: [(0, 0, [3.0, 4.0]), (1, 0, [5.0])], 2: [(0, 0, [6.0, 7.0]), (1, 0, [8.0])]}
    # rank 1 (fast): its round-0 copies -> the reduces fire at 2 copies
    h.scatter(1, 0, 0, [0.0, 1.0])
    assert reduces(h) == [(1, 0, 0, 2, [0.0, 2.0]), (2, 0, 0, 2, [0.0, 2.0])]
    h.scatter(1, 1, 0, [2.0])
    assert reduces(h) == [(1, 1, 0, 2, [4.0]), (2, 1, 0, 2, [4.0])]
    h.reduce(1, 0, 0, 2, [11.0, 11.0])  # one reduced chunk of round 0, then rank 1 moves on
    h.start(basic(9, 1))  # the master starts round 1 while round 0 is open
    h.scatter(1, 0, 1, [10.0, 11.0])  # rank 1's round 1, early
    h.scatter(1, 1, 1, [12.0])
    h.reduce(1, 0, 1, 2, [21.0, 21.0])
    h.reduce(1, 1, 1, 2, [22.0])
    # round 0 has own 2 + 1 = 3 < 4 reduced chunks; round 1 is not served yet
    assert h.take_sent() == [] and h.outputs == []
    # rank 2 (slow): its round-0 copies (outdated: the reduces fired) and one reduced chunk
    h.scatter(2, 0, 0, [0.0, 1.0])
    h.scatter(2, 1, 0, [2.0])
    h.reduce(2, 0, 0, 2, [31.0, 31.0])
    assert [o[0] for o in h.outputs] == [0, 1]  # in order, round 1 right behind round 0
    assert h.outputs[0] == (0, [0.0, 2.0, 4.0, 11.0, 11.0, 0.0, 31.0, 31.0, 0.0], [2, 2, 2, 2, 2, 0, 2, 2, 0],
                            "threshold")
    assert h.outputs[1] == (1, [11.0, 13.0, 15.0, 21.0, 21.0, 22.0, 0.0, 0.0, 0.0], [2, 2, 2, 2, 2, 2, 0, 0, 0],
                            "threshold")
    # round 1 went out only once it was served: its scatters, then its
    # reduces over own + rank 1's early copy (count 2)
    sc = per_dest(h.take_sent("scatter"))
    assert {d: [(m[2], m[3], m[5]) for m in v] for d, v in sc.items()} == \
        {1: [(0, 1, [4.0, 5.0]), (1, 1, [6.0])], 2: [(0, 1, [7.0, 8.0]), (1, 1, [9.0])]}
    red = per_dest(h.take_sent("gather"))
    assert {d: [(m[2], m[3], m[4], m[5]) for m in v] for d, v in red.items()} == \
        {d: [(0, 1, 2, [11.0, 13.0]), (1, 1, 2, [15.0])] for d in (1, 2)}
    h.reduce(2, 1, 0, 2, [32.0])  # round 0 complete: outdated
    assert len(h.outputs) == 2 and h.stats(2)["gather_outdated"] == 1
    assert h.stats(2)["scatter_outdated"] == 2


def test_t8_nasty_chunk_size():
    """SPEC:240-284 (N=2, S=6, C=2, thR 0.9 -> 1, thC 0.8 -> 3): both chunks
    of the worker's block reduce on the first copy (count 1, W:177-181);
    the round completes at the third reduced chunk; a missing chunk is 0 with
    count 0; the late ReduceBlock is outdated."""
    h = SpecHarness(2, 6, 2, 0.9, 0.8, 5)
    h.start(basic(6, 0))
    assert reduces(h) == [(1, 0, 0, 1, [0.0, 1.0]), (1, 1, 0, 1, [2.0])]
    h.scatter(1, 0, 0, [0.0, 1.0])  # after the reduce fired: no new reduce
    h.scatter(1, 1, 0, [2.0])
    assert reduces(h) == []
    assert h.outputs == []
    h.reduce(1, 0, 0, 1, [6.0, 8.0])  # own 2 chunks + this one = floor(0.8 * 4)
    assert h.outputs == [(0, [0.0, 1.0, 2.0, 6.0, 8.0, 0.0], [1, 1, 1, 1, 1, 0], "threshold")]
    h.reduce(1, 1, 0, 1, [10.0])  # after completion: outdated (W:155-156)
    assert len(h.outputs) == 1 and h.stats(1)["gather_outdated"] == 1
    assert h.stats(1)["scatter_outdated"] == 2


def test_t9_nasty_chunk_size_contd():
    """SPEC:286-349 (N=3, S=9, C=1, thR 0.7 -> 2, thC 0.7 -> 6): each chunk
    reduces at its second copy ([0], [2], [4], count 2, to every peer), the
    round completes at 6 of 9 reduced chunks, later chunks are ignored."""
    h = SpecHarness(3, 9, 1, 0.7, 0.7, 5)
    h.start(basic(9, 0))
    assert reduces(h) == []  # own copies only: 1 < 2
    for k in range(3):
        h.scatter(1, k, 0, [float(k)])
    want = [(d, k, 0, 2, [2.0 * k]) for k in range(3) for d in (1, 2)]
    assert reduces(h) == want
    for k in range(3):
        h.scatter(2, k, 0, [float(k)])
    assert reduces(h) == []
    for k, v in enumerate([9.0, 12.0, 15.0]):
        h.reduce(1, k, 0, 2, [v])
    assert [o[0] for o in h.outputs] == [0]  # 3 own + 3 = floor(0.7 * 9)
    for k, v in enumerate([18.0, 21.0, 24.0]):
        h.reduce(2, k, 0, 2, [v])
    assert h.outputs[0][1:3] == ([0.0, 2.0, 4.0, 9.0, 12.0, 15.0, 0.0, 0.0, 0.0], [2, 2, 2, 2, 2, 2, 0, 0, 0])
    assert len(h.outputs) == 1


def test_t10_multi_round():
    """SPEC:351-385 (N=4, S=8, C=2, thR 0.8 -> 3, thC 0.5 -> 2), 10 rounds:
    reduce at the third copy = 3 x [i, 1+i] with count 3; complete at the
    second reduced chunk; later ReduceBlocks of the round are outdated."""
    h = SpecHarness(4, 8, 2, 0.8, 0.5, 5)
    for i in range(10):
        h.start(basic(8, i))
        h.scatter(1, 0, i, [0.0 + i, 1.0 + i])
        assert reduces(h) == []
        h.scatter(2, 0, i, [0.0 + i, 1.0 + i])
        assert reduces(h) == [(d, 0, i, 3, [3.0 * i, 3.0 + 3 * i]) for d in (1, 2, 3)]
        h.scatter(3, 0, i, [0.0 + i, 1.0 + i])
        assert reduces(h) == []
        h.reduce(1, 0, i, 3, [1.0, 2.0])
        assert h.outputs[-1] == (i, [3.0 * i, 3.0 + 3 * i, 1.0, 2.0, 0.0, 0.0, 0.0, 0.0], [3, 3, 3, 3, 0, 0, 0, 0],
                                 "threshold")
        h.reduce(2, 0, i, 3, [1.0, 2.0])
        h.reduce(3, 0, i, 3, [1.0, 2.0])
        assert len(h.outputs) == i + 1 and reduces(h) == []


def test_t11_multi_round_v2():
    """SPEC:387-422 (N=2, S=8, C=2, thR 0.6 -> 1, thC 0.8 -> 3): both own
    chunks reduce on the worker's own copy; complete at 3 of 4."""
    h = SpecHarness(2, 8, 2, 0.6, 0.8, 5)
    for i in range(10):
        h.start(basic(8, i))
        assert reduces(h) == [(1, 0, i, 1, [0.0 + i, 1.0 + i]), (1, 1, i, 1, [2.0 + i, 3.0 + i])]
        h.scatter(1, 0, i, [10.0 + i, 11.0 + i])
        h.scatter(1, 1, i, [12.0 + i, 13.0 + i])
        h.reduce(1, 0, i, 1, [1.0, 2.0])
        assert h.outputs[-1][:3] == (i, [0.0 + i, 1.0 + i, 2.0 + i, 3.0 + i, 1.0, 2.0, 0.0, 0.0],
                                     [1, 1, 1, 1, 1, 1, 0, 0])
        h.reduce(1, 1, i, 1, [1.0, 2.0])
        assert len(h.outputs) == i + 1


def test_t12_missed_scatter():
    """SPEC:424-459 (N=4, S=4, C=2, thR 0.75 -> 3, thC 0.75 -> 3): nothing at
    the second copy, the reduce fires exactly at the third ([0+2+4] = 6,
    count 3); the fourth scatter and the fourth ReduceBlock change nothing."""
    h = SpecHarness(4, 4, 2, 0.75, 0.75, 5)
    h.start(basic(4, 0))
    h.scatter(1, 0, 0, [2.0])
    assert reduces(h) == []
    h.scatter(2, 0, 0, [4.0])
    assert reduces(h) == [(d, 0, 0, 3, [6.0]) for d in (1, 2, 3)]
    h.scatter(3, 0, 0, [6.0])
    assert reduces(h) == [] and h.stats(3)["scatter_outdated"] == 1
    h.reduce(1, 0, 0, 3, [11.0])
    assert h.outputs == []
    h.reduce(2, 0, 0, 3, [10.0])
    assert h.outputs == [(0, [6.0, 11.0, 10.0, 0.0], [3, 3, 3, 0], "threshold")]
    h.reduce(3, 0, 0, 3, [9.0])
    assert len(h.outputs) == 1 and h.stats(3)["gather_outdated"] == 1


def test_t13_future_scatter():
    """SPEC:461-513 (N=4, S=4, C=2, 0.75 / 0.75): a future round's scatter
    arrives while round 0 is still open and waits in round 1's ring row;
    round 0 reduces at its third copy (own [0] + [2] + [4] = 6, count 3),
    the delayed round-0 copy is outdated, round 0 completes at the third
    reduced chunk, then round 1 reduces at ITS third copy (own [1] + 6 + 2).
    (Each peer here makes its round-0 pushes before its round-1 ones: a
    rank's call for round r+1 starts after its call for round r ended.)"""
    h = SpecHarness(4, 4, 2, 0.75, 0.75, 5)
    h.start(basic(4, 0))
    h.scatter(1, 0, 0, [2.0])
    assert reduces(h) == []
    h.scatter(2, 0, 0, [4.0])
    assert reduces(h) == [(d, 0, 0, 3, [6.0]) for d in (1, 2, 3)]
    h.reduce(1, 0, 0, 3, [11.0])
    h.start(basic(4, 1))  # the master starts round 1 (queued: round 0 still open)
    h.scatter(3, 0, 1, [6.0])  # round 1's copy, early: waits in its row
    h.scatter(3, 0, 0, [0.0])  # the delayed round-0 copy: outdated
    assert reduces(h) == [] and h.outputs == [] and h.stats(3)["scatter_outdated"] == 1
    h.reduce(2, 0, 0, 3, [10.0])  # round 0: own + 2 reduced chunks = 3
    assert h.outputs[0] == (0, [6.0, 11.0, 10.0, 0.0], [3, 3, 3, 0], "threshold")
    assert reduces(h) == []  # round 1 served: own + rank 3's copy = 2 < 3
    h.scatter(1, 0, 1, [2.0])
    assert reduces(h) == [(d, 0, 1, 3, [9.0]) for d in (1, 2, 3)]
    h.scatter(2, 0, 1, [4.0])
    for s_, v in ((1, 11.0), (2, 10.0)):
        h.reduce(s_, 0, 1, 3, [v])
    assert h.outputs[1] == (1, [9.0, 11.0, 10.0, 0.0], [3, 3, 3, 0], "threshold")


def test_t14_missed_reduce():
    """SPEC:515-548 (N=4, S=4, C=100, thR 1, thC 0.75): the reduce needs all
    four copies (12, count 4); the round completes with 3 of 4 reduced
    chunks, the missing one 0 with count 0."""
    h = SpecHarness(4, 4, 100, 1.0, 0.75, 5)
    h.start(basic(4, 0))
    for s, v in ((1, 2.0), (2, 4.0)):
        h.scatter(s, 0, 0, [v])
        assert reduces(h) == []
    h.scatter(3, 0, 0, [6.0])
    assert reduces(h) == [(d, 0, 0, 4, [12.0]) for d in (1, 2, 3)]
    h.reduce(1, 0, 0, 4, [11.0])
    assert h.outputs == []
    h.reduce(2, 0, 0, 4, [10.0])
    assert h.outputs == [(0, [12.0, 11.0, 10.0, 0.0], [4, 4, 4, 0], "threshold")]


def test_t15_delayed_future_reduce():
    """SPEC:550-599 (N=4, S=4, C=100, 0.75 / 0.75): ReduceBlocks of rounds 0
    and 1 interleave across peers, in per-pair FIFO order (each peer: its
    round-0 ReduceBlock, then its round-1 messages), so round 0 completes
    before round 1 (SPEC:590)."""
    h = SpecHarness(4, 4, 100, 0.75, 0.75, 5)
    h.start(basic(4, 0))
    h.scatter(1, 0, 0, [2.0])
    h.scatter(2, 0, 0, [4.0])
    assert reduces(h) == [(d, 0, 0, 3, [6.0]) for d in (1, 2, 3)]
    h.scatter(3, 0, 0, [6.0])
    h.start(basic(4, 1))
    h.reduce(1, 0, 0, 3, [11.0])
    h.scatter(1, 0, 1, [3.0])
    h.reduce(1, 0, 1, 3, [11.0])
    assert h.outputs == []
    h.reduce(2, 0, 0, 3, [10.0])  # round 0 complete; round 1 served: own [1] + [3]
    assert [o[0] for o in h.outputs] == [0]
    assert h.outputs[0][1:3] == ([6.0, 11.0, 10.0, 0.0], [3, 3, 3, 0])
    h.scatter(2, 0, 1, [5.0])
    assert reduces(h, 1) == [(d, 0, 1, 3, [9.0]) for d in (1, 2, 3)]
    h.reduce(2, 0, 1, 3, [10.0])
    assert [o[0] for o in h.outputs] == [0, 1]
    assert h.outputs[1][1:3] == ([9.0, 11.0, 10.0, 0.0], [3, 3, 3, 0])
    for m in (("r", 0), ("s", 1), ("r", 1)):  # rank 3, late: all outdated
        if m[0] == "r":
            h.reduce(3, 0, m[1], 3, [9.0])
        else:
            h.scatter(3, 0, m[1], [7.0])
    assert len(h.outputs) == 2 and reduces(h) == []


def test_t16_simple_catchup():
    """SPEC:605-630 (N=4, S=8, C=2, thresholds 1, maxLag 5): rounds stall at
    3 of 4 copies (here rank 3's copies never come; the spec withholds the
    worker's own).  Once a peer is at round 6 > 0 + maxLag, round 0 is
    force-reduced with the copies that landed (count 3) and force-completed
    (W:100-106); rounds 1 and 2 follow at rounds 7 and 8."""
    h = SpecHarness(4, 8, 2, 1.0, 1.0, 5)
    h.start(basic(8, 0))
    for i in range(6):
        for s in (1, 2):
            h.scatter(s, 0, i, [s * (i + 1.0)] * 2)
            h.reduce(s, 0, i, 3, [12.0, 12.0])
    assert h.outputs == [] and reduces(h) == []
    for n, catch in enumerate((6, 7, 8)):
        for s in (1, 2):
            h.scatter(s, 0, catch, [s * (catch + 1.0)] * 2)
            h.reduce(s, 0, catch, 3, [12.0, 12.0])
        i = n
        own = [0.0 + i, 1.0 + i]
        want = [own[0] + 3 * (i + 1), own[1] + 3 * (i + 1)]
        assert reduces(h, i) == [(d, 0, i, 3, want) for d in (1, 2, 3)]
        r, data, counts, reason = h.outputs[-1]
        assert (r, reason) == (i, "catch_up")
        assert data == want + [12.0, 12.0, 12.0, 12.0, 0.0, 0.0] and counts == [3, 3, 3, 3, 3, 3, 0, 0]
        h.start(basic(8, i + 1))  # the worker's next call: round i + 1, still inside the window
    assert h.stats()["reduce_forced"] == 3 and h.stats()["complete_forced"] == 3


def test_t17_cold_catchup():
    """SPEC:632-656: a fresh worker whose peers are at round 10 (maxLag 5)
    starts at round 5 -- the oldest round still inside the window.  The
    reference force-completes rounds 0-4 with zeros / count 0 and then
    re-scatters them; the lane counts them as skipped
    and never scatters them (OneSidedAllreduce's data_sink receives those
    empty outputs)."""
    h = SpecHarness(4, 8, 2, 1.0, 1.0, 5)
    for s in (1, 2, 3):
        h.scatter(s, 0, 10, [1.0, 1.0])
    h.start(basic(8, 0))
    sent = h.take_sent("scatter")
    assert sent and {m[3] for m in sent} == {5}
    assert h.stats()["skipped_rounds"] == 5


def test_t2_early_reduce_of_a_future_round():
    """SPEC:113-131 (N=4, S=8, C=2, thR 1, thC 0.8 -> 3): ReduceBlocks of
    round 3 arrive while the worker is at round 0.  They land in round 3's
    row; every peer announced round 3, so rounds 0-2 can get no copy from
    them and end at once (forced, unreachable -- the reference leaves them
    open).  Round 3 completes at the third landed chunk without the
    worker's own chunk, which is then never reduced (T3 below: the round's
    later scatters are outdated, SPEC:133-138)."""
    h = _t2_early_reduce_of_a_future_round()
    assert [o[0] for o in h.outputs] == [0, 1, 2, 3]
    assert [o[3] for o in h.outputs[:3]] == ["unreachable"] * 3
    r, data, counts, reason = h.outputs[3]
    assert reason == "threshold" and data == [0.0, 0.0, 11.0, 10.0, 10.0, 20.0, 9.0, 10.0]
    assert counts == [0, 0, 4, 4, 4, 4, 4, 4]
    assert h.stats()["reduce_abandoned"] == 1


def test_overwrite_handshake_drops_writes_into_a_row_being_read():
    """Ring depth 2: the worker reads round 0's rows while two peers already
    write round 2 into the same rows.  The writers see the worker's read
    announcement and drop the writes (scatter and gather conflicts); the
    worker sees their "writing 2" tags and excludes them -- nothing torn."""
    h = SpecHarness(4, 8, 2, 0.5, 0.5, 5, rows=2)
    h.start(basic(8, 0))  # need 2 copies: waiting for one peer
    h.scatter(1, 0, 2, [100.0, 100.0])  # round 2 -> row 0, being read for round 0
    h.reduce(2, 0, 2, 4, [200.0, 200.0])
    assert h.stats(1)["scatter_conflict"] == 1 and h.stats(2)["gather_conflict"] == 1
    # ranks 1 and 2 are past round 0 (announced round 2): their copies are
    # lost, so the round ends with what landed, never with round-2 bytes
    h.scatter(3, 0, 0, [3.0, 3.0])
    h.reduce(3, 0, 0, 2, [7.0, 7.0])
    r, data, counts, _ = h.outputs[0]
    assert r == 0 and 100.0 not in data and 200.0 not in data
    assert data[:2] == [3.0, 4.0] and counts[:2] == [2, 2]
    assert data[6:8] == [7.0, 7.0] and counts[2:6] == [0, 0, 0, 0]


def test_dropped_write_leaves_no_phantom_for_its_own_round():
    """A write dropped by the overwrite hand-shake must read as LOST when its
    own round comes up in that row, not as "being written".  Ring depth 2,
    exact thresholds: rank 1 writes round 2 into the row the worker is still
    reading for round 0 and drops it (conflict); it never writes that part
    again.  Rank 1 does not move past round 2 (it stops there, as a rank does
    at the end of a job's phase), so only the tag can tell the worker that
    the copy is gone.  When the worker serves round 2 its wait must end on
    what landed (a phantom "writing 2" tag held it until the lane's timeout:
    a 30 s stall of bench config 4 on the CPU, about once in 150 phase ends)."""
    h = SpecHarness(4, 8, 2, 1.0, 1.0, 5, rows=2)
    h.start(basic(8, 0))
    h.scatter(1, 0, 2, [100.0, 100.0])  # round 2 -> row 0 while it is read for round 0: dropped
    assert h.stats(1)["scatter_conflict"] == 1
    for r in (0, 1):  # ranks 2 and 3 deliver everything; rank 1 is past rounds 0 and 1
        if r == 1:
            h.start(basic(8, 1))
        for src in (2, 3):
            h.scatter(src, 0, r, [float(src), float(src)])
        for src in (2, 3):
            h.reduce(src, 0, r, 3, [10.0 * src, 10.0 * src])
        assert len(h.outputs) == r + 1, (r, h.outputs)
    h.start(basic(8, 2))
    for src in (2, 3):
        h.scatter(src, 0, 2, [float(src), float(src)])
    h.reduce(1, 0, 2, 3, [11.0, 11.0])  # rank 1 completes round 2's phase 2 normally
    for src in (2, 3):
        h.reduce(src, 0, 2, 3, [10.0 * src, 10.0 * src])
    assert len(h.outputs) == 3, "round 2 still waits for the dropped copy"
    r, data, counts, _ = h.outputs[2]
    assert r == 2 and 100.0 not in data
    assert data[:2] == [2.0 + 2 + 3, 3.0 + 2 + 3] and counts[:2] == [3, 3]  # own + ranks 2, 3
    assert data[2:4] == [11.0, 11.0] and counts[2:4] == [3, 3]


def test_dropped_gather_write_leaves_no_phantom_either():
    """The gather side of the same rule: rank 2 writes round 2 (its scatter
    copy and its reduced chunk) into the rows the worker still reads for
    round 0, both writes are dropped, and rank 2 never writes them again.
    Serving round 2 the worker reduces without rank 2's copy and completes
    without its chunk (0, count 0) instead of waiting for either."""
    h = SpecHarness(4, 8, 2, 1.0, 1.0, 5, rows=2)
    h.start(basic(8, 0))
    h.scatter(2, 0, 2, [100.0, 100.0])
    h.reduce(2, 0, 2, 4, [200.0, 200.0])
    assert h.stats(2)["scatter_conflict"] == 1 and h.stats(2)["gather_conflict"] == 1
    for r in (0, 1):  # ranks 1 and 3 deliver everything; rank 2 is past rounds 0 and 1
        if r == 1:
            h.start(basic(8, 1))
        for src in (1, 3):
            h.scatter(src, 0, r, [float(src), float(src)])
        for src in (1, 3):
            h.reduce(src, 0, r, 3, [10.0 * src, 10.0 * src])
        assert len(h.outputs) == r + 1, (r, h.outputs)
    h.start(basic(8, 2))
    for src in (1, 3):
        h.scatter(src, 0, 2, [float(src), float(src)])
    for src in (1, 3):
        h.reduce(src, 0, 2, 3, [10.0 * src, 10.0 * src])
    assert len(h.outputs) == 3, "round 2 still waits for a dropped copy"
    r, data, counts, _ = h.outputs[2]
    assert r == 2 and 100.0 not in data and 200.0 not in data
    assert data[:2] == [2.0 + 1 + 3, 3.0 + 1 + 3] and counts[:2] == [3, 3]
    assert data[4:6] == [0.0, 0.0] and counts[4:6] == [0, 0]  # rank 2's block: never arrived


@pytest.mark.parametrize("seed", range(6))
def test_random_orders_match_reference_rules(seed):
    """Random arrival orders of one round's messages (N=4, thresholds 0.75):
    the reduce fires at the third copy over exactly the copies that landed,
    the round completes at floor(0.75 * total) reduced chunks, everything
    after is dropped -- checked against the reference's rules directly."""
    rng = np.random.default_rng(seed)
    N, S, C = 4, 12, 1
    h = SpecHarness(N, S, C, 0.75, 0.75, 5)
    g = h.g
    x = [float(v) for v in rng.integers(-5, 5, S)]
    h.start(x)
    kme = g.num_chunks(0)
    msgs = [("s", s, k) for s in range(1, N) for k in range(kme)]
    msgs += [("r", s, k) for s in range(1, N) for k in range(g.num_chunks(s))]
    rng.shuffle(msgs)
    landed = {k: [0] for k in range(kme)}
    vals = {}
    reduced = {}
    got_reduced = []
    need_c = int(np.float32(0.75) * np.float32(g.total_chunks()))
    for kind, s, k in msgs:
        if h.outputs:
            break
        if kind == "s":
            v = float(rng.integers(1, 9))
            vals[(s, k)] = v
            h.scatter(s, k, 0, [v])
            if k not in reduced:
                landed[k].append(s)
                if len(landed[k]) == 3:
                    reduced[k] = x[g.chunk_offset(0, k)] + sum(vals[(q, k)] for q in landed[k] if q)
        else:
            v = float(100 * s + k)
            h.reduce(s, k, 0, 3, [v])
            got_reduced.append((s, k, v))
        sent = reduces(h)
        for d, k2, _, cnt, vv in sent:
            assert cnt == 3 and vv == [reduced[k2]]
        if len(reduced) + len(got_reduced) >= need_c:
            assert len(h.outputs) == 1
    if h.outputs:
        r, data, counts, reason = h.outputs[0]
        assert reason == "threshold"
        for k, v in reduced.items():
            assert data[g.chunk_offset(0, k)] == v
        for s, k, v in got_reduced:
            assert data[g.chunk_offset(s, k)] == v


def test_t4_t5_partial_membership_then_reinit():
    """SPEC:141-170 (N=4, S=8, C=2, thresholds 1, maxLag 5, worker 0).
    T4: with the peer map {0} the worker scatters only to itself -- no push
    to an absent rank (it is not mapped at all: dead until it joins).  T5: a
    re-InitWorkers with the full map (the windows of ranks 1-3 mapped between
    rounds) and StartAllreduce(1): the worker scatters round 1 to every
    peer, chunk [2i+1, 2i+2] to rank i, rotated from itself.
    By design (docs/DESIGN.md): round 0 cannot reach thReduce = 1 without
    the absent ranks and nothing more can arrive, so it completes at once
    (reason "unreachable") with the worker's own block (count 1) and zeros
    with count 0 elsewhere, where the reference's round would wait forever."""
    h = SpecHarness(4, 8, 2, 1.0, 1.0, 5, members=[0])
    assert h.w.members() == [0]
    h.start(basic(8, 0))
    assert h.take_sent("scatter") == []            # only the self-scatter, delivered in place
    # one chunk per absent peer in each phase (its scatter, then the forced
    # reduce's broadcast), never pushed
    assert h.stats()["dead_skips"] == 6
    assert reduces(h, 0) == []
    assert len(h.outputs) == 1
    rnd, data, cnt, reason = h.outputs[0]
    assert rnd == 0 and reason == "unreachable"
    assert data[:2] == [0.0, 1.0] and cnt[:2] == [1, 1]
    assert data[2:] == [0.0] * 6 and cnt[2:] == [0] * 6
    for q in (1, 2, 3):
        h.admit(q)
    assert h.w.members() == [0, 1, 2, 3]
    h.start(basic(8, 1))
    sc = h.take_sent("scatter")
    assert [(m[1], m[2], m[3], m[5]) for m in sc] == [(i, 0, 1, [2.0 * i + 1, 2.0 * i + 2]) for i in (1, 2, 3)]
    # and the round now waits for the joined ranks' copies (thReduce = 1)
    assert len(h.outputs) == 1
    for src in (1, 2, 3):
        h.scatter(src, 0, 1, [1.0, 2.0])
    red = reduces(h, 1)
    assert [(m[0], m[1], m[3]) for m in red] == [(1, 0, 4), (2, 0, 4), (3, 0, 4)]
    assert red[0][4] == [4.0, 8.0]
    # re-admitting a mapped rank is refused (a departed rank stays dead)
    with pytest.raises(Exception):
        h.admit(1)
