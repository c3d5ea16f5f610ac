"""Differential test: the native engine against the executable specification
in ``model_worker.py``, on random message sequences.

Each example draws a geometry (N, S, C, id), thresholds, maxLag, whether the
worker delivers to itself directly (SPEC T1) or through the probe, and a
random sequence of StartAllreduce / ScatterBlock / ReduceBlock messages --
future rounds, outdated rounds, duplicates, partial thresholds, catch-up.
Every message the worker emits (scatter, reduce, complete, in order) and every
sink output (round, data, per-element counts) must match the model's.
"""
import os

import hypothesis.strategies as st
import pytest
import torch
from hypothesis import HealthCheck, given, settings

from akka_allreduce_amd import AllreduceWorker
from akka_allreduce_amd.messages import (CompleteAllreduce, InitWorkers, ReduceBlock, ScatterBlock, StartAllreduce,
                                         WorkerTerminated)
from akka_allreduce_amd.testing import TestProbe

from model_worker import Geometry, ModelWorker

MAX_ROUND = 8
THRESHOLDS = [0.2, 0.5, 0.6, 0.75, 0.9, 1.0]


def source_values(S, r):
    return [float((i * 3 + r * 5) % 7 - 3) for i in range(S)]


@st.composite
def scenarios(draw):
    N = draw(st.integers(2, 5))
    S = draw(st.integers(1, 24))
    C = draw(st.integers(1, 5))
    me = draw(st.integers(0, N - 1))
    g = Geometry(S, N, C)
    kme = g.num_chunks(me)
    owners = [j for j in range(N) if g.num_chunks(j) > 0]
    val = st.integers(-4, 4).map(float)
    rounds = st.integers(0, MAX_ROUND)
    kinds = ["start", "reduce", "membership"] + (["scatter", "scatter"] if kme > 0 else [])
    subset = st.sets(st.integers(0, N - 1)).map(lambda p: sorted(p | {me}))
    events = []
    for _ in range(draw(st.integers(1, 60))):
        kind = draw(st.sampled_from(kinds))
        if kind == "start":
            events.append(("start", draw(rounds)))
        elif kind == "membership":  # re-InitWorkers with another peer map (T4/T5), or a peer death
            others = [j for j in range(N) if j != me]
            if draw(st.booleans()):
                events.append(("reinit", draw(subset)))
            else:
                events.append(("terminated", draw(st.sampled_from(others))))
        elif kind == "scatter":
            k = draw(st.integers(0, kme - 1))
            vals = draw(st.lists(val, min_size=g.chunk_len(me, k), max_size=g.chunk_len(me, k)))
            events.append(("scatter", draw(st.integers(0, N - 1)), k, draw(rounds), vals))
        else:
            j = draw(st.sampled_from(owners))
            k = draw(st.integers(0, g.num_chunks(j) - 1))
            vals = draw(st.lists(val, min_size=g.chunk_len(j, k), max_size=g.chunk_len(j, k)))
            events.append(("reduce", j, k, draw(rounds), draw(st.integers(0, N)), vals))
    return dict(N=N, S=S, C=C, me=me, peers=draw(subset), max_lag=draw(st.integers(0, 3)), th_reduce=draw(st.sampled_from(THRESHOLDS)),
                th_complete=draw(st.sampled_from(THRESHOLDS)), self_local=draw(st.booleans()), events=events)


def _msg_tuple(m):
    if isinstance(m, ScatterBlock):
        return ("scatter", m.srcId, m.destId, m.chunkId, m.round, [float(v) for v in torch.as_tensor(m.value).tolist()])
    if isinstance(m, ReduceBlock):
        return ("reduce", m.srcId, m.destId, m.chunkId, m.round, m.count,
                [float(v) for v in torch.as_tensor(m.value).tolist()])
    if isinstance(m, CompleteAllreduce):
        return ("complete", m.srcId, m.round)
    raise AssertionError(f"unexpected message {m!r}")


def run_native(sc, device="cpu"):
    S = sc["S"]
    probe = TestProbe()
    sink = []
    w = AllreduceWorker(lambda req: torch.tensor(source_values(S, req.iteration)),
                        lambda o: sink.append((o.iteration, [float(v) for v in o.data.tolist()],
                                               [int(c) for c in o.count.tolist()])),
                        device=device, strict=True)
    def peer_map(ids):
        m = {i: probe for i in ids}
        if sc["self_local"]:
            m[sc["me"]] = w
        return m

    w.tell(InitWorkers(peer_map(sc["peers"]), sc["N"], probe, sc["me"], sc["th_reduce"], sc["th_complete"], sc["max_lag"], S, sc["C"]))
    for ev in sc["events"]:
        if ev[0] == "start":
            w.tell(StartAllreduce(ev[1]))
        elif ev[0] == "reinit":
            w.tell(InitWorkers(peer_map(ev[1]), sc["N"], probe, sc["me"], sc["th_reduce"], sc["th_complete"],
                               sc["max_lag"], S, sc["C"]))
        elif ev[0] == "terminated":
            w.tell(WorkerTerminated(ev[1]))
        elif ev[0] == "scatter":
            _, src, k, r, vals = ev
            w.tell(ScatterBlock(torch.tensor(vals), src, sc["me"], k, r))
        else:
            _, src, k, r, count, vals = ev
            w.tell(ReduceBlock(torch.tensor(vals), src, sc["me"], k, r, count))
    assert not w.errors, w.errors
    return [_msg_tuple(m) for m in probe.drain()], sink


def run_model(sc):
    m = ModelWorker(lambda r: source_values(sc["S"], r), self_local=sc["self_local"])
    m.init(sc["me"], sc["N"], sc["th_reduce"], sc["th_complete"], sc["max_lag"], sc["S"], sc["C"], sc["peers"])
    for ev in sc["events"]:
        if ev[0] == "start":
            m.start(ev[1])
        elif ev[0] == "reinit":
            m.reinit(ev[1])
        elif ev[0] == "terminated":
            m.terminated(ev[1])
        elif ev[0] == "scatter":
            _, src, k, r, vals = ev
            m.on_scatter(src, sc["me"], k, r, vals)
        else:
            _, src, k, r, count, vals = ev
            m.on_reduce(src, sc["me"], k, r, count, vals)
    return m.out, m.sink


EXAMPLES = int(os.environ.get("AKKA_MODEL_EXAMPLES", "400"))
QUIET = [HealthCheck.too_slow, HealthCheck.data_too_large]


def check(sc, device):
    got_msgs, got_sink = run_native(sc, device)
    want_msgs, want_sink = run_model(sc)
    assert got_msgs == want_msgs
    assert got_sink == want_sink


@settings(max_examples=EXAMPLES, deadline=None, suppress_health_check=QUIET)
@given(scenarios())
def test_engine_matches_model(sc):
    check(sc, "cpu")


@pytest.mark.gpu
@settings(max_examples=max(50, EXAMPLES // 4), deadline=None, suppress_health_check=QUIET)
@given(scenarios())
def test_engine_matches_model_on_gpu(sc):
    """Same sequences on the HIP data plane: every chunk sum is the gfx950
    reduce kernel, outputs/counts are bound device tensors."""
    check(sc, "cuda")
