"""The reactive (straggler-tolerant) transport on the CPU p2p simulator.

Same native code as on MI355X (ReactiveLink: one stream per peer, per-pair
grouped p2p, event-polled arrivals, staged data plane); the simulator decides
which ranks' streams advance, so frozen ranks, stragglers and arbitrary
stream interleavings are reproducible.

Inputs are x_i = 2^i * w (w = 1..3 per element), so every output element
reveals exactly which ranks contributed to it: the contributor mask must have
popcount == the delivered count (the reference's count semantics, RB:41-47).
"""
import random

import pytest
import torch

from akka_allreduce_amd.data import Geometry
from akka_allreduce_amd.messages import StartAllreduce
from akka_allreduce_amd.parallel.sim import ReactiveSimCluster


def _w(S):
    return (torch.arange(S) % 3 + 1).float()


def _x(i, S):
    return _w(S) * float(1 << i)


def _check_masks(o, S, n, allowed=None):
    w = _w(S)
    mask = (o.data / w).round().long()
    assert torch.equal(mask.float() * w, o.data), "not a subset sum"
    pc = torch.zeros_like(mask)
    for b in range(n):
        bit = (mask >> b) & 1
        pc += bit
        if allowed is not None and b not in allowed:
            assert int(bit.sum()) == 0, f"rank {b} contributed but should not have"
    assert torch.equal(pc.int(), o.count), "popcount(contributors) != count"
    return mask


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("S,C", [(64, 8), (1000, 7), (778, 3), (5, 1), (333, 1000)])
def test_reactive_exact(n, S, C):
    cl = ReactiveSimCluster(n, S, C, max_lag=1)
    for r in range(3):
        g = torch.Generator().manual_seed(r)
        xs = [torch.randint(-8, 9, (S,), generator=g).float() for _ in range(n)]
        for i in range(n):
            cl.start(i, xs[i])
        cl.run(lambda: all(cl.done(i, r) for i in range(n)))
        cl.settle()
        want = torch.stack(xs).sum(0)
        for i in range(n):
            o = cl.outputs[i][r]
            assert torch.equal(o.data, want), (i, r)
            assert bool((o.count == n).all())
    cl.drain()
    for w in cl.workers:
        st = w.state()
        assert st["round"] == 3 and st["link"]["in_flight"] == 0 and st["link"]["slots_busy"] == 0


def test_reactive_bf16():
    n, S, C = 4, 999, 50
    cl = ReactiveSimCluster(n, S, C, dtype=torch.bfloat16)
    xs = [torch.randint(-8, 9, (S,)).bfloat16() for _ in range(n)]
    for i in range(n):
        cl.start(i, xs[i])
    cl.run(lambda: all(cl.done(i, 0) for i in range(n)))
    cl.settle()
    want = torch.stack([x.float() for x in xs]).sum(0).bfloat16()
    assert all(torch.equal(cl.outputs[i][0].data, want) for i in range(n))


def test_frozen_rank_does_not_stall_the_others():
    """thReduce = thComplete = 0.75, rank 3 frozen: ranks 0-2 complete every
    round from their own three contributions (the reference's core promise)."""
    n, S, C, R = 4, 64, 4, 6
    cl = ReactiveSimCluster(n, S, C, th_reduce=0.75, th_complete=0.75, max_lag=2)
    fast = [0, 1, 2]
    for r in range(R):
        for i in fast:
            cl.start(i, _x(i, S))
        cl.run(lambda: all(cl.done(i, r) for i in fast), active=fast)
    cl.settle(fast)
    g = Geometry(S, n, C)
    s3, e3 = g.block_range(3)
    for i in fast:
        for r in range(R):
            o = cl.outputs[i][r]
            mask = _check_masks(o, S, n, allowed={0, 1, 2})
            assert bool((mask[:s3] == 0b111).all())
            assert bool((o.count[s3:e3] == 0).all())  # rank 3's block never reduced
    st = cl.workers[0].state()["link"]
    assert st["slots_busy"] == R  # one pinned send slot per round the frozen peer owes
    # the straggler wakes up and runs the same rounds: everything drains
    for r in range(R):
        cl.start(3, _x(3, S))
    cl.run(lambda: all(cl.done(3, r) for r in range(R)))
    cl.settle()
    for r in range(R):
        _check_masks(cl.outputs[3][r], S, n)
    cl.drain()
    assert all(w.state()["link"]["slots_busy"] == 0 for w in cl.workers)
    assert all(w.round == R for w in cl.workers)


def test_slow_rank_interleaved():
    """A rank whose streams advance only every 5th step: exact thresholds still
    give exact results; partial thresholds let the others run ahead."""
    n, S, C = 4, 200, 16
    for th in (1.0, 0.75):
        cl = ReactiveSimCluster(n, S, C, th_reduce=th, th_complete=th, max_lag=3, seed=7)
        started = [0] * n
        R = 6
        tick = 0
        while not all(cl.done(i, R - 1) for i in range(n)):
            tick += 1
            active = [0, 1, 2] + ([3] if tick % 5 == 0 else [])
            for i in active:
                # a rank starts its next round once its previous one completed
                if started[i] < R and (started[i] == 0 or cl.done(i, started[i] - 1)):
                    cl.start(i, _x(i, S))
                    started[i] += 1
            cl.step(active, shuffle=True)
            assert tick < 20000
        cl.settle()
        for i in range(n):
            for r in range(R):
                mask = _check_masks(cl.outputs[i][r], S, n)
                if th == 1.0:
                    assert bool((mask == 0b1111).all())
        cl.drain()


@pytest.mark.parametrize("seed", range(6))
def test_random_interleavings(seed):
    """Random stream interleavings and random per-step rank freezes."""
    rng = random.Random(seed)
    n = rng.choice([2, 3, 4, 5])
    S = rng.choice([17, 100, 257])
    C = rng.choice([1, 4, 9, 64])
    th = rng.choice([1.0, 0.75, 0.6])
    cl = ReactiveSimCluster(n, S, C, th_reduce=th, th_complete=th, max_lag=rng.choice([1, 2, 3]), seed=seed)
    R = 5
    started = [0] * n
    steps = 0
    while not all(cl.done(i, R - 1) for i in range(n)):
        steps += 1
        assert steps < 50000, "no progress"
        active = [i for i in range(n) if rng.random() < 0.7] or [rng.randrange(n)]
        for i in active:
            if started[i] < R and (started[i] == 0 or cl.done(i, started[i] - 1)):
                cl.start(i, _x(i, S))
                started[i] += 1
        cl.step(active, shuffle=True)
    cl.settle()
    for i in range(n):
        for r in range(R):
            mask = _check_masks(cl.outputs[i][r], S, n)
            if th == 1.0:
                assert bool((mask == (1 << n) - 1).all())
    cl.drain()


def test_cold_catch_up():
    """A rank that was frozen receives StartAllreduce far ahead (master
    pacing): it force-completes the rounds it missed (W:100-106), re-scatters
    them for slower peers, and the pair streams stay aligned."""
    n, S, C, lag = 4, 48, 4, 1
    cl = ReactiveSimCluster(n, S, C, th_reduce=0.75, th_complete=0.75, max_lag=lag)
    fast = [0, 1, 2]
    R = 4
    for r in range(R):
        for i in fast:
            cl.start(i, _x(i, S))
        cl.run(lambda: all(cl.done(i, r) for i in fast), active=fast)
    w3 = cl.workers[3]
    for r in range(R):  # inputs for every round it will fetch
        w3._feed[r] = _x(3, S)
    w3._next_round = R
    w3.receive(StartAllreduce(R - 1))
    cl._collect(3)
    st = w3.state()["stats"]
    assert st["rounds_forced"] >= R - 1 - lag
    cl.run(lambda: all(cl.done(3, r) for r in range(R)))
    cl.settle()
    for r in range(R):
        _check_masks(cl.outputs[3][r], S, n)
    # afterwards everyone runs full rounds together again
    for r in range(R, R + 2):
        for i in range(n):
            cl.start(i, _x(i, S))
        cl.run(lambda: all(cl.done(i, r) for i in range(n)))
    cl.settle()
    for i in range(n):
        for r in range(R, R + 2):
            _check_masks(cl.outputs[i][r], S, n)
    cl.drain()
    assert all(w.state()["link"]["slots_busy"] == 0 for w in cl.workers)


def test_slot_pool_exhaustion_is_bounded_wait_not_error():
    """More rounds than send slots while a peer is frozen: the oldest finished
    round's slot is reclaimed by a stream wait, so the fast ranks stall
    (bounded staleness) until the frozen rank wakes -- then everything drains."""
    n, S, C = 3, 30, 5
    cl = ReactiveSimCluster(n, S, C, th_reduce=0.6, th_complete=0.6, max_lag=1)
    fast = [0, 1]
    done_rounds = 0
    for r in range(40):
        for i in fast:
            cl.start(i, _x(i, S))
        try:
            cl.run(lambda: all(cl.done(i, r) for i in fast), active=fast, max_idle=20)
        except RuntimeError:
            break
        done_rounds = r + 1
    slots = cl.workers[0].state()["link"]["slots"]
    assert done_rounds >= slots - 2, (done_rounds, slots)
    assert done_rounds < 40
    # wake rank 2: it catches up, all pending transfers complete
    for r in range(done_rounds + 1):
        cl.start(2, _x(2, S))
    cl.run(lambda: all(cl.done(2, r) for r in range(done_rounds + 1)))
    cl.run(lambda: all(cl.done(i, done_rounds) for i in fast))
    cl.settle()
    cl.drain()


@pytest.mark.parametrize("n", range(2, 17))
def test_pair_communicator_tournament(n):
    """The ncclCommSplit schedule that builds one RCCL communicator per pair:
    each round is a matching, every unordered pair meets exactly once."""
    from akka_allreduce_amd._native_loader import load

    rounds = load().tournament(n)
    met = set()
    for partner in rounds:
        for x, p in enumerate(partner):
            if p >= n:
                continue
            assert p != x and partner[p] == x  # symmetric matching
            met.add((min(x, p), max(x, p)))
    assert met == {(a, b) for a in range(n) for b in range(a + 1, n)}
    assert len(rounds) == (n if n % 2 else n - 1)


def test_threshold_allreduce_reactive_guards():
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    with pytest.raises(ValueError):
        ThresholdAllreduce(16, transport="bogus", rank=0, world_size=1, device="cpu")
    # N = 1 needs no peers: the local path serves both transports
    ar = ThresholdAllreduce(16, transport="reactive", rank=0, world_size=1, device="cpu")
    o = ar(torch.arange(16.0))
    assert torch.equal(o.data, torch.arange(16.0))


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_small_pool_freezes_and_thresholds(seed, monkeypatch):
    """Random freezes with a tiny send-slot pool (reclaim by stream wait),
    random thresholds/lag/geometry: every round of every rank completes, the
    contributor-mask/count invariant holds, nothing stays in flight."""
    rng = random.Random(1000 + seed)
    monkeypatch.setenv("AKKA_REACTIVE_SLOTS", str(rng.choice([2, 3, 4])))
    # transfer groups of 1 chunk, a few chunks, or whole blocks
    monkeypatch.setenv("AKKA_REACTIVE_GROUP_BYTES", str(rng.choice([0, 24, 100, 1 << 24])))
    n = rng.choice([2, 3, 4])
    S = rng.choice([9, 64, 130])
    C = rng.choice([1, 5, 16, 200])
    th = rng.choice([1.0, 0.75, 0.5])
    lag = rng.choice([1, 2])
    cl = ReactiveSimCluster(n, S, C, th_reduce=th, th_complete=th, max_lag=lag, seed=seed)
    R = 8
    started = [0] * n
    frozen_until = [0] * n
    for step in range(200000):
        if all(cl.done(i, R - 1) for i in range(n)):
            break
        if rng.random() < 0.02:
            v = rng.randrange(n)
            frozen_until[v] = step + rng.randrange(5, 200)
        active = [i for i in range(n) if frozen_until[i] <= step] or [rng.randrange(n)]
        for i in active:
            if started[i] < R and (started[i] == 0 or cl.done(i, started[i] - 1)):
                cl.start(i, _x(i, S))
                started[i] += 1
        cl.step(active, shuffle=True)
    else:
        raise AssertionError("fuzz run did not finish")
    cl.settle()
    for i in range(n):
        for r in range(R):
            mask = _check_masks(cl.outputs[i][r], S, n)
            if th == 1.0:
                assert bool((mask == (1 << n) - 1).all())
    cl.drain()
    assert all(w.state()["link"]["in_flight"] == 0 for w in cl.workers)


def _dead_rank_run(n, dead, S, C, rounds, warm, slots, monkeypatch, th=0.75):
    monkeypatch.setenv("AKKA_REACTIVE_SLOTS", str(slots))
    from akka_allreduce_amd.messages import WorkerTerminated

    cl = ReactiveSimCluster(n, S, C, th_reduce=th, th_complete=th, max_lag=1)
    alive = [i for i in range(n) if i != dead]
    for r in range(warm):  # everyone together first
        for i in range(n):
            cl.start(i, _x(i, S))
        cl.run(lambda: all(cl.done(i, r) for i in range(n)))
    # `dead` stops for good; the survivors keep starting rounds until the
    # send-slot pool would stall them, then the control plane reports the death
    told = False
    for r in range(warm, warm + rounds):
        for i in alive:
            cl.start(i, _x(i, S))
        try:
            cl.run(lambda: all(cl.done(i, r) for i in alive), active=alive, max_idle=30)
        except RuntimeError:
            assert not told, f"survivors stalled at round {r} after the death was reported"
            for i in alive:
                cl.workers[i].receive(WorkerTerminated(dead))
            told = True
            cl.run(lambda: all(cl.done(i, r) for i in alive), active=alive)
    cl.settle(alive)
    return cl, alive, told


@pytest.mark.parametrize("warm", [0, 3])
def test_dead_peer_survivors_keep_going(warm, monkeypatch):
    """A rank that dies for good (never steps again): once the survivors are
    told (WorkerTerminated, the reference's Terminated handler W:141-146 made
    reachable), their transfers with it are aborted and forgotten, so they
    complete far more rounds than the send-slot pool holds (the pool would
    otherwise park them on the dead rank forever).  Its contributions are
    missing: no output element ever contains it afterwards, and the block it
    owned arrives as zeros with count 0."""
    n, dead, S, C, slots = 4, 3, 64, 8, 4
    rounds = 2 * slots + 4
    cl, alive, told = _dead_rank_run(n, dead, S, C, rounds, warm, slots, monkeypatch)
    assert told  # without the report the pool would have stalled them
    g = Geometry(S, n, C)
    s3, e3 = g.block_range(dead)
    for i in alive:
        for r in range(warm + 2, warm + rounds):  # rounds after the death settled
            o = cl.outputs[i][r]
            _check_masks(o, S, n, allowed=set(alive))
            assert int(o.count[s3:e3].abs().sum()) == 0  # its block: zeros, count 0
            assert bool((o.count[:s3] <= n - 1).all())
        st = cl.workers[i].state()["link"]
        assert st["peers_lost"] == 1
    cl.drain(alive)
    assert all(cl.workers[i].state()["link"]["in_flight"] == 0 for i in alive)


def test_dead_peer_reported_up_front_never_exchanged(monkeypatch):
    """Told before the first round: nothing is ever posted to the dead rank."""
    from akka_allreduce_amd.messages import WorkerTerminated

    monkeypatch.setenv("AKKA_REACTIVE_SLOTS", "3")
    n, S, C = 4, 40, 5
    cl = ReactiveSimCluster(n, S, C, th_reduce=0.75, th_complete=0.75, max_lag=1)
    alive = [0, 1, 2]
    for i in alive:
        cl.workers[i].receive(WorkerTerminated(3))
    for r in range(10):
        for i in alive:
            cl.start(i, _x(i, S))
        cl.run(lambda: all(cl.done(i, r) for i in alive), active=alive)
    cl.settle(alive)
    for i in alive:
        for r in range(10):
            _check_masks(cl.outputs[i][r], S, n, allowed=set(alive))
    assert cl.workers[0].state()["link"]["transfers_dropped"] == 0


def test_partial_membership_islands_reactive():
    """T4/T5 across real ranks on the reactive transport: two islands {0,1}
    and {2,3} exchange only within themselves, then a re-InitWorkers with the
    full map (at a round boundary) makes every pair exchange."""
    import random as _random

    from akka_allreduce_amd._native_loader import load
    from akka_allreduce_amd.worker import AllreduceWorker

    import tests.test_sim_schedule as ts

    n, S, C = 4, 64, 4
    cl = ReactiveSimCluster.__new__(ReactiveSimCluster)
    cl._nat = load()
    cl.n = n
    cl.hub = cl._nat.SimHub(n)
    cl.rng = _random.Random(0)
    cl.workers = [AllreduceWorker(None, None, device="cpu", transport="reactive", transport_spec=("sim", cl.hub, r),
                                  strict=True, name=f"risl{r}") for r in range(n)]
    cl.outputs = [dict() for _ in range(n)]
    rounds = [0]

    def run_round(xs):
        r = rounds[0]
        for i in range(n):
            cl.start(i, xs[i])
        cl.run(lambda: all(cl.done(i, r) for i in range(n)))
        cl.settle()
        cl.drain()
        rounds[0] += 1
        return [cl.outputs[i][r] for i in range(n)]

    ts._islands(cl, n, S, C, 0.5, run_round, chunk_order=False)
    # round 0: phase 1 from the one island peer; round 1: from all three
    # (4 chunks per block, one arrival per chunk and peer; which chunks make
    # the 50% is timing)
    k = Geometry(S, n, C).num_chunks(0)
    for w in cl.workers:
        st = w.state()["link"]
        assert st["p1_arrivals"] == k * (1 + 3) and st["p2_arrivals"] == k * (1 + 3), st


def test_chunk_granular_phase2_overlaps_phase1(monkeypatch):
    """maxChunkSize is the transfer unit (W:218-232): every chunk is its own
    P1 / P2 exchange, and a chunk is broadcast the moment it is reduced
    (W:177-181) -- chunk 0's phase-2 groups go out while later phase-1 chunks
    of the same round are still in flight (phase 2 has its own pair channel,
    so it never queues behind them)."""
    monkeypatch.setenv("AKKA_REACTIVE_GROUP_BYTES", "0")  # one chunk per transfer group
    n, S, C = 3, 3 * 8 * 16, 16  # 8 chunks per block
    cl = ReactiveSimCluster(n, S, C, max_lag=1)
    xs = [torch.randint(-8, 9, (S,), generator=torch.Generator().manual_seed(i)).float() for i in range(n)]
    for i in range(n):
        cl.start(i, xs[i])
    cl.run(lambda: all(cl.done(i, 0) for i in range(n)))
    cl.settle()
    want = torch.stack(xs).sum(0)
    for i in range(n):
        assert torch.equal(cl.outputs[i][0].data, want)
        st = cl.workers[i].state()["link"]
        assert st["p2_overlapped"] > 0, st
        assert st["p1_arrivals"] == (n - 1) * 8 and st["p2_arrivals"] == (n - 1) * 8
    cl.drain()


@pytest.mark.parametrize("group_bytes", ["0", "128", "1000000"])
@pytest.mark.parametrize("th", [1.0, 0.67])
def test_transfer_groups_any_size(group_bytes, th, monkeypatch):
    """Transfer groups of 1, 2 and all chunks (fixed bounds from the
    geometry): same sums / contributor counts, every chunk delivered once."""
    monkeypatch.setenv("AKKA_REACTIVE_GROUP_BYTES", group_bytes)
    n, S, C = 3, 3 * 7 * 16 + 5, 16  # 7-8 chunks per block, short last chunk
    cl = ReactiveSimCluster(n, S, C, th_reduce=th, th_complete=th, max_lag=1)
    for r in range(3):
        for i in range(n):
            cl.start(i, _x(i, S))
        cl.run(lambda: all(cl.done(i, r) for i in range(n)))
    cl.settle()
    for i in range(n):
        for r in range(3):
            mask = _check_masks(cl.outputs[i][r], S, n)
            if th == 1.0:
                assert bool((mask == (1 << n) - 1).all())
    cl.drain()
