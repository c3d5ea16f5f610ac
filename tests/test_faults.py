"""Fault injection utilities (utils/faults.py) against the message-driven
engine: duplicated messages never double-count (fire-once, distinct
sources), dropped messages leave count-0 holes but rounds still complete at
thresholds < 1, delayed messages arrive out of order and are still placed."""
import time

import torch

from akka_allreduce_amd.messages import InitWorkers, ReduceBlock, ScatterBlock, StartAllreduce
from akka_allreduce_amd.parallel.actors import LocalSystem
from akka_allreduce_amd.utils.faults import FaultyRef, env_straggler_delay, straggler_source
from akka_allreduce_amd.worker import AllreduceWorker


def _cluster(n, S, C, th, fault):
    sys_ = LocalSystem()
    outs = [dict() for _ in range(n)]
    ws = []
    for i in range(n):
        def sink(o, i=i):
            outs[i][o.iteration] = (o.data.clone(), o.count.clone())
        ws.append(AllreduceWorker(lambda req, i=i: torch.full((S,), float(1 << i)), sink, device="cpu",
                                  name=f"f{i}"))
    refs = [sys_.spawn(w, f"w{i}") for i, w in enumerate(ws)]
    for i, w in enumerate(ws):
        peers = {j: (refs[j] if j == i else fault(j, refs[j])) for j in range(n)}
        w.tell(InitWorkers(peers, n, None, i, th, th, 1, S, C))
    return sys_, ws, refs, outs


def test_duplicates_never_double_count():
    n, S, C = 4, 40, 3
    faults = []

    def fault(j, ref):
        f = FaultyRef(ref, dup=0.5, seed=j)
        faults.append(f)
        return f

    sys_, ws, refs, outs = _cluster(n, S, C, 1.0, fault)
    for r in range(3):
        for ref in refs:
            sys_.post(ref, StartAllreduce(r))
        sys_.run()
    assert sum(f.stats.duplicated for f in faults) > 0
    for i in range(n):
        for r in range(3):
            data, count = outs[i][r]
            assert torch.equal(data, torch.full((S,), 15.0)) and bool((count == 4).all())


def test_drops_leave_holes_but_rounds_complete():
    n, S, C = 4, 64, 4
    faults = []

    def fault(j, ref):
        f = FaultyRef(ref, drop=0.15, seed=100 + j)
        faults.append(f)
        return f

    sys_, ws, refs, outs = _cluster(n, S, C, 0.5, fault)
    for r in range(4):
        for ref in refs:
            sys_.post(ref, StartAllreduce(r))
        sys_.run()
    assert sum(f.stats.dropped for f in faults) > 0
    done = 0
    for i in range(n):
        for r, (data, count) in outs[i].items():
            done += 1
            mask = data.round().long()
            pc = sum(((mask >> b) & 1) for b in range(n))
            assert torch.equal(pc.int(), count)  # every element: value's contributor set == count
    assert done >= n * 3


def test_delays_reorder_but_results_exact():
    n, S, C = 3, 30, 4
    faults = []

    def fault(j, ref):
        f = FaultyRef(ref, delay_s=lambda m: 0.002 * (hash((m.chunkId, m.round)) % 5), seed=j)
        faults.append(f)
        return f

    sys_, ws, refs, outs = _cluster(n, S, C, 1.0, fault)
    for ref in refs:
        sys_.post(ref, StartAllreduce(0))
    t0 = time.time()
    while any(0 not in o for o in outs) and time.time() - t0 < 10:
        sys_.run()
        time.sleep(0.005)
    for i in range(n):
        data, count = outs[i][0]
        assert torch.equal(data, torch.full((S,), 7.0)) and bool((count == 3).all())


def test_straggler_source_and_env(monkeypatch):
    calls = []
    src = straggler_source(lambda req: calls.append(req) or 1, 0.01, rounds=lambda r: r % 2 == 0)

    class Req:
        iteration = 0

    t0 = time.perf_counter()
    src(Req())
    assert time.perf_counter() - t0 >= 0.009
    monkeypatch.setenv("AKKA_FAULT_RANK", "2")
    monkeypatch.setenv("AKKA_FAULT_DELAY_MS", "25")
    assert env_straggler_delay(2) == 0.025 and env_straggler_delay(1) == 0.0
