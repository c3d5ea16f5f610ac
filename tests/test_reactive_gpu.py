"""Reactive transport on one MI355X: N ranks in one process, each with its
own HIP streams (one per peer), staged data plane and ReactiveLink, over the
asynchronous per-pair loopback (device copies released by stream
write-value).  Checks exact sums at thresholds 1, the contributor-mask/count
invariant at partial thresholds, and that a sleeping rank does not stall the
others (then catches up)."""
import pytest
import torch

from akka_allreduce_amd.data import Geometry
from akka_allreduce_amd.parallel.loopback import ReactiveLoopbackCluster

pytestmark = pytest.mark.gpu


def _w(S):
    return (torch.arange(S, device="cuda") % 3 + 1).float()


def _check_masks(o, S, n, allowed=None):
    w = _w(S)
    mask = (o.data.float() / w).round().long()
    assert torch.equal(mask.float() * w, o.data.float())
    pc = torch.zeros_like(mask)
    for b in range(n):
        bit = (mask >> b) & 1
        pc += bit
        if allowed is not None and b not in allowed:
            assert int(bit.sum()) == 0
    assert torch.equal(pc.int(), o.count)
    return mask


@pytest.mark.parametrize("n", [2, 3, 4])
@pytest.mark.parametrize("S,C", [(1 << 16, 1 << 12), (100_003, 777), (5, 1)])
def test_reactive_loopback_exact(n, S, C):
    with ReactiveLoopbackCluster(n, S, C, max_lag=1) as cl:
        _exact(cl, n, S)


def _exact(cl, n, S):
    rounds = []
    for k in range(4):
        g = torch.Generator().manual_seed(k)
        rounds.append([torch.randint(-8, 9, (S,), generator=g).float().cuda() for _ in range(n)])
    outs = cl.run_rounds(rounds)
    torch.cuda.synchronize()
    for k, xs in enumerate(rounds):
        want = torch.stack(xs).sum(0)
        for r in range(n):
            assert torch.equal(outs[r][k].data, want), (n, S, k, r)
            assert bool((outs[r][k].count == n).all())


def test_reactive_loopback_bf16():
    n, S, C = 3, 300_001, 4096
    with ReactiveLoopbackCluster(n, S, C, dtype=torch.bfloat16) as cl:
        xs = [torch.randint(-8, 9, (S,)).bfloat16().cuda() for _ in range(n)]
        outs = cl.run_rounds([xs])
        want = torch.stack([x.float() for x in xs]).sum(0).bfloat16()
        torch.cuda.synchronize()
        assert all(torch.equal(outs[r][0].data, want) for r in range(n))


def test_reactive_loopback_sleeping_rank():
    """Rank 3 sleeps 3 s; at thresholds 0.75 ranks 0-2 finish all rounds long
    before it wakes, summing only each other's data; then rank 3 catches up.

    Runs in a fresh child process: its ranks' 20 streams must each get a
    hardware queue of their own.  In the suite's process, streams of earlier
    tests can push a fast rank's stream onto a queue shared with a stream
    parked on the sleeper, and that fast rank then waits for the sleeper (a
    harness artefact: one process per GPU on a node)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-c", "import test_reactive_gpu as t; t._sleeping_child()"], cwd=here,
                       env=dict(os.environ, GPU_MAX_HW_QUEUES="32",
                                PYTHONPATH=os.pathsep.join([os.path.dirname(here), here,
                                                            os.environ.get("PYTHONPATH", "")])),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "sleeping ok" in r.stdout, r.stdout[-2000:]


def _sleeping_child():
    n, S, C, R = 4, 1 << 14, 1 << 10, 4
    cl = ReactiveLoopbackCluster(n, S, C, th_reduce=0.75, th_complete=0.75, max_lag=2)
    try:
        _sleeping(cl, n, S, C, R)
    finally:
        cl.close()
    print("sleeping ok", flush=True)


def _sleeping(cl, n, S, C, R):
    import time

    rounds = [[_w(S) * float(1 << i) for i in range(n)] for _ in range(R)]
    done_at = {}
    orig = cl.workers[0].allreduce

    t0 = time.monotonic()

    def timed(x, **kw):
        o = orig(x, **kw)
        done_at[o.iteration] = time.monotonic() - t0
        return o

    cl.workers[0].allreduce = timed
    outs = cl.run_rounds(rounds, delays=[0, 0, 0, 3.0])
    torch.cuda.synchronize()
    assert max(done_at.values()) < 2.5, done_at  # never waited for the sleeper
    g = Geometry(S, n, C)
    s3, _ = g.block_range(3)
    for r in range(3):
        for k in range(R):
            mask = _check_masks(outs[r][k], S, n, allowed={0, 1, 2})
            assert bool((mask[:s3] == 0b111).all())
    for k in range(R):
        _check_masks(outs[3][k], S, n)
    cl.drain()
    assert all(w.state()["link"]["slots_busy"] == 0 for w in cl.workers)


def test_reactive_loopback_dead_peer(monkeypatch):
    """Rank 3 is gone for good (never posts).  The survivors are told after
    two rounds (WorkerTerminated): their pair transfers with it are aborted
    (pair loopback: both directions released, queued posts dropped) and they
    run far more rounds than the 4-slot send pool holds, summing only each
    other's data; rank 3's block arrives as zeros with count 0."""
    import threading

    from akka_allreduce_amd.messages import WorkerTerminated

    monkeypatch.setenv("AKKA_REACTIVE_SLOTS", "4")
    n, S, C, R = 4, 1 << 14, 1 << 10, 12
    cl = ReactiveLoopbackCluster(n, S, C, th_reduce=0.75, th_complete=0.75, max_lag=1)
    alive = [0, 1, 2]
    outs = {r: [] for r in alive}
    errs = []

    def run(r):
        try:
            w = cl.workers[r]
            w.reactive_timeout = 30.0
            for k in range(R):
                if k == 2:
                    w.receive(WorkerTerminated(3))
                outs[r].append(w.allreduce(_w(S) * float(1 << r)))
            torch.cuda.current_stream().synchronize()
        except BaseException as e:  # pragma: no cover - surfaced below
            errs.append(e)

    ts = [threading.Thread(target=run, args=(r,)) for r in alive]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    try:
        assert not errs, errs
        g = Geometry(S, n, C)
        s3, e3 = g.block_range(3)
        for r in alive:
            assert len(outs[r]) == R
            for k in range(R):
                o = outs[r][k]
                _check_masks(o, S, n, allowed=set(alive))
                assert int(o.count[s3:e3].abs().sum()) == 0
            st = cl.workers[r].state()["link"]
            assert st["peers_lost"] == 1
        for r in alive:
            cl.workers[r].synchronize()
    finally:
        cl.hub.release_all()
        for w in cl.workers:
            w.close()
