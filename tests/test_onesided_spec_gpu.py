"""The reference spec's arrival orders replayed against the REAL gfx950 round
kernel: every case of tests/test_onesided_spec.py runs
unchanged with ``WindowSpecHarness`` in place of its CPU harness.

``AllreduceSpec.scala`` drives one real worker and plays every peer (and the
master) with the TestKit probe (SPEC:812-818).  Here the worker is rank 0's
``OneSidedLane`` on the GPU: each ``start`` enqueues one call of
``os_round_kernel`` on the worker's stream, and the kernel's roles (push,
decide, reduce, complete, copy) run on the card while the test plays the
peers: ``inject`` performs a peer's push from the host into the worker's
device window -- through the same gates and tags a peer kernel uses -- while
the worker's kernel spins in its waits.  All N lanes live in this one process
(same-process windows need no IPC mapping); only the worker ever launches.

The worker's own pushes land in the peers' (passive) windows, where the
harness reads them back as the probe reads the worker's messages: a "done r"
tag of a part is one message of round r, its bytes and count word the
payload.  The messages pending at a look are ordered the way the CPU harness
emits them (round, scatter before reduce, chunk, part, peers rotated from the
worker), so every assertion of the CPU cases -- outputs
``(round, data, counts, reason)``, emitted messages, counters -- holds
verbatim on the device.  After every step the harness waits for the card to
go quiet (no new output and no new message for a few polls), which is what
the spec's ``expectNoMsg`` does with its timeout.

``device=-1`` runs the same harness on CPU lanes (begin / progress), which
checks the harness itself without a GPU (tests/test_onesided_spec.py keeps
its own held-outbox harness)."""
from __future__ import annotations

import inspect
import time

import numpy as np
import pytest
import torch

import test_onesided_spec as spec
from akka_allreduce_amd._native_loader import load
from model_worker import Geometry

_OPEN: list = []  # harnesses of the running test (closed after it: every launched call must end)
_STREAMS: dict = {}  # the worker's and the copy stream, created once (streams share hardware queues)


def _streams(dev):
    if dev not in _STREAMS:
        _STREAMS[dev] = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    return _STREAMS[dev]


class WindowSpecHarness:
    """Drop-in for test_onesided_spec.SpecHarness on device lanes."""

    device = 0
    quiet_polls = 3
    poll_s = 0.015
    max_settle_s = 2.0

    def __init__(self, N, S, C, th_reduce, th_complete, max_lag, me=0, rows=0, members=None, window_output=False):
        nat = load()
        self.N, self.S, self.C, self.me = N, S, C, me
        self.g = Geometry(S, N, C)
        self.kmax = max(1, max(self.g.num_chunks(j) for j in range(N)))
        dev = self.device
        self.lanes = [nat.OneSidedLane(dev, S, N, C, r, "float32", th_reduce=th_reduce, th_complete=th_complete,
                                       max_lag=max_lag, rows=rows, part_bytes=1 << 40,
                                       timeout_ms=20_000 if dev >= 0 else 3_600_000,
                                       window_output=window_output and dev >= 0)
                      for r in range(N)]
        hs = [ln.handle() for ln in self.lanes]
        self.handles = hs
        for r, ln in enumerate(self.lanes):
            if r == me and members is not None:
                ln.open([h if q in members or q == me else b"" for q, h in enumerate(hs)])
            else:
                ln.open(hs)
        self.w = self.lanes[me]
        info = self.w.info()
        self.D, self.P = int(info["rows"]), int(info["parts"])
        assert self.P == 1  # one part per chunk: a message of the spec is one chunk
        self.tags = self.D * N * self.kmax * self.P
        self.outputs: list = []
        self.sent: list = []
        self._seen: set = set()
        self.calls: list = []  # in flight, in order
        self.cur = None        # CPU lanes: the call begin() started
        self.pending: list = []
        if dev >= 0:
            self.cuda = torch.device("cuda", dev)
            self.stream, self.copy_stream = _streams(self.cuda)
            # first-time work of the runtime (side streams, staging buffers
            # for pageable copies) may wait for the whole device: done here,
            # before any call is in flight, not in the middle of a round
            for ln in self.lanes:
                ln.peek_flags()
                ln.peek_part(0, 0, 0, 0, 0)
                ln.stats_nowait()
            with torch.cuda.stream(self.copy_stream):
                torch.zeros(4, device=self.cuda).cpu()
            torch.cuda.synchronize(self.cuda)
        _OPEN.append(self)

    # ---- layout (csrc/kernels/onesided_protocol.h, Layout::init) -----------------
    def _stag(self, row, src, k, j=0):
        return 2 * (((row * self.N + src) * self.kmax + k) * self.P + j)

    def _gtag(self, row, blk, k, j=0):
        return 2 * self.tags + self._stag(row, blk, k, j)

    # ---- the worker ---------------------------------------------------------------
    def start(self, data):
        """The worker's next call (StartAllreduce from the master, M:83-89)."""
        x = torch.tensor([float(v) for v in data], dtype=torch.float32)
        out = torch.full((self.S,), float("nan"))
        counts = torch.full((self.N, self.kmax), -1, dtype=torch.int32)
        if self.device < 0:
            self.pending.append((x, out, counts))
        else:
            # the buffers are staged on the copy stream: a blocking copy on the
            # worker's stream would wait for the call still running there
            with torch.cuda.stream(self.copy_stream):
                x, out, counts = (t.to(self.cuda, non_blocking=False) for t in (x, out, counts))
            self.stream.wait_stream(self.copy_stream)
            for t in (x, out, counts):
                t.record_stream(self.stream)
            with torch.cuda.stream(self.stream):
                call = self.w.round(self.stream.cuda_stream, x.data_ptr(), out.data_ptr(), counts.data_ptr(),
                                    self.kmax)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.calls.append((x, out, counts, call, ev))
        self.settle()

    def _finish(self, out, counts, call):
        st = self.w.status(call)
        per_el = [0] * self.S
        for j in range(self.N):
            for k in range(self.g.num_chunks(j)):
                o = self.g.chunk_offset(j, k)
                for e in range(o, o + self.g.chunk_len(j, k)):
                    per_el[e] = int(counts[j, k])
        self.outputs.append((st["round"], [float(v) for v in out.tolist()], per_el, st["reason"]))

    def pump(self):
        if self.device < 0:
            while True:
                if self.cur is None and self.pending:
                    x, out, counts = self.pending.pop(0)
                    call = self.w.begin(x.data_ptr(), out.data_ptr(), counts.data_ptr(), self.kmax)
                    self.cur = (x, out, counts, call)
                if self.cur is None or not self.w.progress():
                    break
                self._finish(self.cur[1], self.cur[2], self.cur[3])
                self.cur = None
        else:
            while self.calls and self.calls[0][4].query():
                x, out, counts, call, ev = self.calls.pop(0)
                with torch.cuda.stream(self.copy_stream):
                    self.copy_stream.wait_event(ev)
                    oc, cc = out.cpu(), counts.cpu()
                self._finish(oc, cc, call)
        self._collect()

    def _collect(self):
        """The worker's pushes that landed in the peers' windows since the last look."""
        new = []
        for q in range(self.N):
            if q == self.me:
                continue
            fl = self.lanes[q].peek_flags()
            for phase in (0, 1):
                nch = self.g.num_chunks(q if phase == 0 else self.me)
                for row in range(self.D):
                    for k in range(nch):
                        w = self._stag(row, self.me, k) if phase == 0 else self._gtag(row, self.me, k)
                        t = int(fl[w])
                        if t < 3 or t % 2 == 0:
                            continue  # nothing yet / a write in progress
                        r = (t - 1) // 2 - 1
                        key = (phase, q, k, r)
                        if key in self._seen:
                            continue
                        self._seen.add(key)
                        vals = np.frombuffer(self.lanes[q].peek_part(phase, row, self.me, k, 0),
                                             dtype=np.float32).tolist()
                        cnt = int(fl[w + 1]) if phase == 1 else 0
                        new.append(("scatter" if phase == 0 else "gather", q, k, r, cnt, vals))
        self.sent.extend(new)

    def _sig(self):
        return len(self.outputs), len(self._seen), len(self.calls), self.cur is not None, len(self.pending)

    def settle(self):
        """Step until the worker is quiet: no new output / message for a few polls."""
        self.pump()
        if self.device < 0:
            return
        last, quiet, t_end = self._sig(), 0, time.monotonic() + self.max_settle_s
        while quiet < self.quiet_polls and time.monotonic() < t_end:
            time.sleep(self.poll_s)
            self.pump()
            s = self._sig()
            quiet = quiet + 1 if s == last else 0
            last = s

    def take_sent(self, phase=None):
        # everything pending since the test's last look is one step for the
        # test: order it as the CPU harness emits (the device publishes the
        # parts of one decision to the peers in any order, and a look may
        # fall between them)
        self.sent.sort(key=lambda m: (m[3], 0 if m[0] == "scatter" else 1, m[2], (m[1] - self.me - 1) % self.N))
        s = [m for m in self.sent if phase is None or m[0] == phase]
        self.sent = [m for m in self.sent if not (phase is None or m[0] == phase)]
        return s

    def admit(self, q):
        self.w.add_peer(q, self.handles[q])

    # ---- the peers ------------------------------------------------------------------
    def scatter(self, src, k, r, vals):
        self.lanes[src].inject(0, self.me, k, 0, r, 0, np.asarray(vals, dtype=np.float32).tobytes())
        self.settle()

    def reduce(self, src, k, r, count, vals):
        self.lanes[src].inject(1, self.me, k, 0, r, count, np.asarray(vals, dtype=np.float32).tobytes())
        self.settle()

    def stats(self, rank=None):
        return self.lanes[self.me if rank is None else rank].stats_nowait()

    def close(self):
        """End every launched call (force all waits) and drain the device."""
        self.w.force_below(1 << 31)
        if self.device >= 0:
            self.stream.synchronize()
            self.copy_stream.synchronize()
            torch.cuda.synchronize(self.cuda)


class CpuWindowSpecHarness(WindowSpecHarness):
    device = -1


def window_catchup_waits_for_held_writer():
    """Window output: the result of a call is the gather row of
    its CALL id.  A call that caught up serves another round, in another row,
    and must not return a row a peer is still writing.  Replayed on the GPU
    kernel with a peer whose gather push of round 1 (row 1) passed its gate
    before call 1 began and stores its bytes only after the call's own round
    (2, row 0) has fully landed: call 1 waits for that writer before it
    writes its result into row 1, so the late bytes can never land on top of
    it.  N=2, S=8, C=2 (two chunks of 2 per block), thresholds 1, maxLag 1."""
    from torch.utils.dlpack import from_dlpack

    N, S, C = 2, 8, 2
    h = WindowSpecHarness(N, S, C, 1.0, 1.0, 1, rows=2, window_output=True)
    try:
        w, peer = h.w, h.lanes[1]
        assert w.info()["window_output"], w.info()
        rows = [from_dlpack(w.gather_row_dlpack(d, "float32", h.device)) for d in range(h.D)]
        f32 = lambda v: np.asarray(v, dtype=np.float32).tobytes()  # noqa: E731

        def call(xv):
            with torch.cuda.stream(h.stream):
                x = torch.tensor(xv, dtype=torch.float32, device=h.cuda)
                counts = torch.full((N, h.kmax), -1, dtype=torch.int32, device=h.cuda)
                c = w.round(h.stream.cuda_stream, x.data_ptr(), 0, counts.data_ptr(), h.kmax)
                ev = torch.cuda.Event()
                ev.record(h.stream)
            return x, counts, c, ev

        def wait(ev, s=10.0):
            t_end = time.monotonic() + s
            while not ev.query():
                assert time.monotonic() < t_end, "the call did not finish"
                time.sleep(0.005)

        def result(c, counts):
            with torch.cuda.stream(h.copy_stream):
                return rows[c % h.D].cpu().tolist(), counts.cpu().tolist(), w.status(c)

        # round 0, call 0 -> row 0
        x0 = [1.0] * S
        t0 = call(x0)
        for k in range(2):
            peer.inject(0, 0, k, 0, 0, 0, f32([10.0, 10.0]))        # peer's copy of my block
            peer.inject(1, 0, k, 0, 0, 2, f32([7.0, 7.0]))          # block 1 reduced
        wait(t0[3])
        d0, n0, st0 = result(t0[2], t0[1])
        assert st0["round"] == 0 and d0 == [11.0] * 4 + [7.0] * 4, (st0, d0)
        # a peer's gather push of round 1 into row 1 passes its gate, then stalls
        peer.inject(1, 0, 0, 0, 1, 2, f32([999.0, 999.0]), stage=1)
        # the peer moves on to round 3: call 1 catches up to round 2 (lo = 3 - maxLag)
        peer.inject(0, 0, 0, 0, 3, 0, f32([0.0, 0.0]))
        x1 = [2.0] * S
        t1 = call(x1)   # call id 1 -> its result is row 1; the round it serves lives in row 0
        for k in range(2):
            peer.inject(0, 0, k, 0, 2, 0, f32([20.0, 20.0]))
            peer.inject(1, 0, k, 0, 2, 2, f32([5.0, 5.0]))
        time.sleep(0.2)
        assert not t1[3].query(), "call 1 must wait for the writer still storing into its result row"
        peer.inject(1, 0, 0, 0, 1, 2, f32([999.0, 999.0]), stage=2)   # the stalled bytes land now
        wait(t1[3])
        d1, n1, st1 = result(t1[2], t1[1])
        assert st1["round"] == 2, st1
        assert d1 == [22.0] * 4 + [5.0] * 4, d1          # not a 999 in it
        assert all(v == 2 for r_ in n1 for v in r_), n1
        assert w.error() == 0
    finally:
        h.close()
        _OPEN.remove(h) if h in _OPEN else None


EXTRA = {"window_catchup_waits_for_held_writer": window_catchup_waits_for_held_writer}

CASES = sorted(name for name, f in inspect.getmembers(spec, inspect.isfunction)
               if name.startswith("test_") and "seed" not in inspect.signature(f).parameters)
SEEDS = range(4)


def run_case(name, harness, seed=None):
    """One case of tests/test_onesided_spec.py with ``harness`` as its SpecHarness."""
    saved = spec.SpecHarness
    spec.SpecHarness = harness
    try:
        f = getattr(spec, name)
        f(seed) if seed is not None else f()
    finally:
        spec.SpecHarness = saved
        while _OPEN:
            _OPEN.pop().close()


@pytest.mark.parametrize("name", CASES)
def test_spec_case_on_window_harness_cpu(name):
    """The harness itself on CPU lanes: the same assertions hold when the
    worker's pushes are delivered to (and read back from) the peers' windows."""
    run_case(name, CpuWindowSpecHarness)


@pytest.fixture(scope="module")
def gpu_results():
    """Every case on the GPU in ONE child process with GPU_MAX_HW_QUEUES=16:
    the harness's copy stream and the lanes' host-side stream must not share
    a hardware queue with the worker's stream, where a copy would queue behind
    the round kernel it is meant to observe (4 queues by default)."""
    import json
    import os
    import subprocess
    import sys
    import tempfile

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    here = os.path.dirname(os.path.abspath(__file__))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "results.json")
        env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
        r = subprocess.run([sys.executable, os.path.join(here, "spec_gpu_runner.py"), out], cwd=os.path.dirname(here),
                           env=env, capture_output=True, text=True, timeout=900)
        assert os.path.exists(out), (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
        return json.load(open(out))


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_spec_case_on_gpu_kernel(name, gpu_results):
    res = gpu_results[name]
    assert res["ok"], res["error"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_spec_random_orders_on_gpu_kernel(seed, gpu_results):
    res = gpu_results[f"random_orders_{seed}"]
    assert res["ok"], res["error"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(EXTRA))
def test_window_case_on_gpu_kernel(name, gpu_results):
    res = gpu_results[name]
    assert res["ok"], res["error"]
