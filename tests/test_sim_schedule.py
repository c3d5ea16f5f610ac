"""The RCCL/xGMI step schedule, N = 2..8 ranks, on the CPU p2p simulator.

Checks exact sums and counts, multi-round pipelining through the ring,
uneven/empty blocks, bf16, thresholds < 1 (deterministic arrival order in the
scheduled transport), traffic volume = the direct algorithm's 2(N-1)/N * S
per rank, and that a schedule mismatch between ranks is caught (deadlock /
size mismatch) instead of hanging.
"""
import pytest
import torch

from akka_allreduce_amd.data import Geometry
from akka_allreduce_amd.parallel.sim import SimCluster


def _inputs(n, S, r, dtype=torch.float32):
    g = torch.Generator().manual_seed(100 * r + n)
    # small integers: sums are exact in fp32 and bf16
    return [torch.randint(-8, 9, (S,), generator=g).to(dtype) for _ in range(n)]


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("S,C", [(64, 8), (1000, 7), (778, 3), (5, 1), (4096, 4096), (333, 1000)])
def test_exact_sum_all_ranks(n, S, C):
    cl = SimCluster(n, S, C, max_lag=1)
    for r in range(3):
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        for rank, o in enumerate(outs):
            assert o.iteration == r
            assert torch.equal(o.data, want), (rank, r)
            assert bool((o.count == n).all()), (rank, r)
    for w in cl.workers:
        st = w.state()
        assert st["round"] == 3 and st["stats"]["rounds_completed"] == 3


@pytest.mark.parametrize("lag", [1, 2, 3])
def test_broadcast_lag_variants(lag, monkeypatch):
    monkeypatch.setenv("AKKA_EXACT_UNIT_BYTES", "0")  # one chunk per step
    n, S, C = 4, 4096, 100
    cl = SimCluster(n, S, C, broadcast_lag=lag)
    xs = _inputs(n, S, 0)
    outs = cl.allreduce(xs)
    want = torch.stack(xs).sum(0)
    assert all(torch.equal(o.data, want) for o in outs)
    g = Geometry(S, n, C)
    assert cl.workers[0].state()["link"]["groups"] == g.kmax + lag


def test_bf16():
    n, S, C = 8, 10_000, 256
    cl = SimCluster(n, S, C, dtype=torch.bfloat16)
    xs = _inputs(n, S, 0, torch.bfloat16)
    outs = cl.allreduce(xs)
    want = torch.stack([x.float() for x in xs]).sum(0).bfloat16()
    assert all(torch.equal(o.data, want) for o in outs)


def test_traffic_volume_matches_direct_algorithm():
    """Exact rounds move exactly the direct algorithm's payload (every count
    is N by construction: no counts exchange); threshold rounds also carry
    each owner's per-chunk counts (the ReduceBlock.count field)."""
    n, S, C = 8, 8192, 128
    g = Geometry(S, n, C)
    payload = 2 * (n - 1) * S * 4  # each rank: (N-1)/N*S out in phase 1 and phase 2
    counts = sum((n - 1) * g.num_chunks(j) * 4 for j in range(n))  # each owner -> N-1 peers
    cl = SimCluster(n, S, C)
    cl.allreduce(_inputs(n, S, 0))
    assert cl.bytes_moved() == payload
    assert cl.workers[0].state()["link"]["exact_step_rounds"] == 1
    cl = SimCluster(n, S, C, th_reduce=0.99)
    cl.allreduce(_inputs(n, S, 0))
    assert cl.bytes_moved() == payload + counts
    assert cl.workers[0].state()["link"]["exact_step_rounds"] == 0


def test_many_rounds_ring_reuse():
    n, S, C = 3, 300, 16
    cl = SimCluster(n, S, C, max_lag=0)  # one ring row: every round reuses it
    for r in range(12):
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        assert all(torch.equal(o.data, want) for o in outs), r


def test_threshold_reduce_subset_is_deterministic():
    """thReduce < 1: each owner reduces the first floor(th*N) arrivals, which in
    the scheduled transport are itself then peers me+1, me+2, ... (rotation)."""
    n, S, C = 4, 400, 50
    th = 0.75  # -> 3 of 4
    cl = SimCluster(n, S, C, th_reduce=th)
    xs = _inputs(n, S, 0)
    outs = cl.allreduce(xs)
    g = Geometry(S, n, C)
    m = 3
    want = torch.zeros(S)
    for j in range(n):
        s, e = g.block_range(j)
        srcs = [(j + i) % n for i in range(m)]
        want[s:e] = torch.stack([xs[q][s:e] for q in srcs]).sum(0)
    for o in outs:
        assert torch.equal(o.data, want)
        assert bool((o.count == m).all())


def test_mismatched_schedule_is_detected(monkeypatch):
    # uneven chunks (8,8,8,6 per block): a rank with a different broadcast lag
    # issues its per-pair ops in a different order -> a size mismatch, not silent corruption
    monkeypatch.setenv("AKKA_EXACT_UNIT_BYTES", "0")
    n, S, C = 2, 60, 8
    cl = SimCluster(n, S, C, broadcast_lag=[1, 2])
    xs = _inputs(n, S, 0)
    with pytest.raises(RuntimeError, match="sim p2p"):
        cl.allreduce(xs)


@pytest.mark.parametrize("n,S,C,th", [(3, 63 * 4, 4, 0.67), (4, 64 * 4, 4, 0.5), (8, 320, 5, 0.6), (3, 252, 4, 0.8)])
def test_completion_before_late_chunks_are_reduced(n, S, C, th):
    """thComplete < 1 with many chunks per block: the round completes while
    later chunks are still ahead in the schedule; scatters for them are then
    outdated (W:172-173), so they are never reduced, yet the symmetric
    schedule must still send something at their broadcast step -- zeros with
    count 0.  Every element's value must be a subset sum whose contributor
    count equals the delivered count (inputs are 2^rank)."""
    cl = SimCluster(n, S, C, th_reduce=th, th_complete=th)
    for r in range(3):
        outs = cl.allreduce([torch.full((S,), float(1 << i)) for i in range(n)])
        for o in outs:
            m = o.data.round().long()
            pc = sum(((m >> b) & 1) for b in range(n))
            assert torch.equal(pc.int(), o.count)
            assert bool((o.count == 0).any())  # some chunks never made it: holes, not garbage
    assert cl.workers[0].state()["link"]["unreduced_chunks"] > 0


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("S,C", [(64, 8), (1000, 7), (5, 1), (4096, 4096), (333, 1000)])
def test_collective_lane_exact(n, S, C):
    """Exact rounds on the whole-round lane (stream_link.cpp bulk_round): the
    simulator has no native collectives, so this is the whole-block direct
    exchange -- two grouped p2p per round around one N-way reduce.  Same sums
    and counts as the chunk schedule, traffic = 2(N-1)/N*S per rank, no
    separate counts exchange (every count is N)."""
    cl = SimCluster(n, S, C, max_lag=1, lane="collective")
    g = Geometry(S, n, C)
    before = 0
    for r in range(4):
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        for rank, o in enumerate(outs):
            assert o.iteration == r
            assert torch.equal(o.data, want), (rank, r)
            assert bool((o.count == n).all()), (rank, r)
        moved = cl.bytes_moved() - before
        before = cl.bytes_moved()
        assert moved == 2 * (n - 1) * S * 4
    for w in cl.workers:
        st = w.state()
        assert st["round"] == 4 and st["stats"]["rounds_completed"] == 4
        assert st["stats"]["bulk_rounds"] == 4 and st["link"]["bulk_rounds"] == 4
        assert st["link"]["groups"] == 4 * 2 and st["link"]["lane"] == "collective"
        assert st["stats"]["chunks_reduced"] == 4 * g.num_chunks(st["id"])


def test_collective_lane_only_for_exact_rounds():
    """Thresholds < 1 depend on arrival order: the lane is not taken."""
    n, S, C = 4, 400, 50
    cl = SimCluster(n, S, C, th_reduce=0.75, lane="collective")
    cl.allreduce(_inputs(n, S, 0))
    assert all(w.state()["link"]["bulk_rounds"] == 0 for w in cl.workers)
    assert all(w.state()["link"]["exact_step_rounds"] == 0 for w in cl.workers)


def test_auto_lane_without_native_collectives_keeps_chunk_schedule(monkeypatch):
    monkeypatch.setenv("AKKA_EXACT_UNIT_BYTES", "0")
    n, S, C = 4, 4096, 100
    cl = SimCluster(n, S, C)
    cl.allreduce(_inputs(n, S, 0))
    st = cl.workers[0].state()
    assert st["link"]["collective_rounds"] == 0 and st["link"]["lane"] == "auto"
    assert st["link"]["exact_step_rounds"] == 1
    assert st["link"]["groups"] == Geometry(S, n, C).kmax + 2


def test_lane_switch_between_rounds():
    n, S, C = 3, 999, 10
    cl = SimCluster(n, S, C, max_lag=2)
    for r, lane in enumerate(["p2p", "collective", "p2p", "collective", "collective"]):
        for w in cl.workers:
            w.set_lane(lane)
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        assert all(torch.equal(o.data, want) and bool((o.count == n).all()) for o in outs), (r, lane)
    st = cl.workers[0].state()["link"]
    assert st["bulk_rounds"] == 5 and st["exact_step_rounds"] == 2


def _islands(cl, n, S, C, th, run_round, chunk_order=True):
    """T4/T5 across real ranks: start as two islands {0,1} and {2,3} (each
    rank's InitWorkers lists only its island, SPEC:141-162), then a
    re-InitWorkers with the full map at a round boundary (W:87-89,
    SPEC:164-170).  Inputs 2^rank reveal who contributed to each element."""
    from akka_allreduce_amd.messages import InitWorkers
    from akka_allreduce_amd.parallel.collective import _RemoteRank

    isl = {0: [0, 1], 1: [0, 1], 2: [2, 3], 3: [2, 3]}
    for r, w in enumerate(cl.workers):
        peers = {i: (w if i == r else _RemoteRank(i)) for i in isl[r]}
        w.tell(InitWorkers(peers, n, None, r, th, th, 1, S, C))
    xs = [torch.full((S,), float(1 << i)) for i in range(n)]
    outs0 = run_round(xs)
    g = Geometry(S, n, C)
    for r, o in enumerate(outs0):
        for j in range(n):
            s, e = g.block_range(j)
            if j in isl[r]:  # my island's blocks: reduced from the island only
                want = float(sum(1 << i for i in isl[r]))
                assert torch.equal(o.data[s:e], torch.full((e - s,), want)), (r, j)
                assert bool((o.count[s:e] == 2).all())
            else:  # the other island's blocks never reach me: zeros, count 0
                assert int(o.count[s:e].abs().sum()) == 0 and int(o.data[s:e].abs().sum()) == 0
    for r, w in enumerate(cl.workers):  # re-init: the full map (only the peers change)
        peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
        w.tell(InitWorkers(peers, n, None, r, th, th, 1, S, C))
    outs1 = run_round(xs)
    for r, o in enumerate(outs1):
        got = o.count > 0
        # thReduce 0.5: reduced from the first two arrivals; thComplete 0.5:
        # the round completes with half of the chunks, the rest read 0/0
        assert bool((o.count[got] == 2).all())
        m = o.data.long()[got]
        assert bool(((m & (m - 1)) != 0).all())  # two distinct contributors
        if chunk_order:  # scheduled transport: every block's first chunk arrives first
            for j in range(n):
                s, _ = g.block_range(j)
                assert int(o.count[s]) == 2, (r, j)
    return outs0, outs1


def test_partial_membership_islands_stream_transport():
    n, S, C = 4, 64, 4
    hub_before = []
    cl = SimCluster.__new__(SimCluster)
    from akka_allreduce_amd._native_loader import load
    from akka_allreduce_amd.worker import AllreduceWorker

    cl.n = n
    cl.hub = load().SimHub(n)
    cl.workers = [AllreduceWorker(None, None, device="cpu", transport="stream", transport_spec=("sim", cl.hub, r),
                                  strict=True, name=f"isl{r}") for r in range(n)]

    def run_round(xs):
        hub_before.append(cl.bytes_moved())
        return cl.allreduce(xs)

    _islands(cl, n, S, C, 0.5, run_round)
    # round 0 moved island traffic only; round 1 the full direct volume
    r0 = cl.bytes_moved() - hub_before[1]
    assert hub_before[1] < r0


def test_lone_member_completes_from_itself():
    """Every other worker gone (peer map = {me}), thresholds 0.5: my block is
    reduced from my own contribution and delivered -- not mistaken for an
    unreduced chunk because nobody needs its broadcast."""
    from akka_allreduce_amd._native_loader import load
    from akka_allreduce_amd.messages import InitWorkers
    from akka_allreduce_amd.worker import AllreduceWorker

    hub = load().SimHub(2)
    w = AllreduceWorker(None, None, device="cpu", transport="stream", transport_spec=("sim", hub, 0), strict=True)
    S, C = 4096, 256
    w.tell(InitWorkers({0: w}, 2, None, 0, 0.5, 0.5, 1, S, C))
    for r in range(3):
        x = torch.full((S,), float(r + 3))
        o = w.allreduce(x)
        load().sim_run(hub, [w._core])
        assert torch.equal(o.data[:S // 2], x[:S // 2]) and bool((o.count[:S // 2] == 1).all())
        assert int(o.count[S // 2:].abs().sum()) == 0
    assert w.state()["link"]["unreduced_chunks"] == 0


@pytest.mark.parametrize("unit_bytes", ["0", "800", "1200", str(16 << 20)])
@pytest.mark.parametrize("n,S,C", [(4, 4096, 100), (3, 1000, 7), (8, 8192 + 5, 64)])
def test_exact_transfer_units(unit_bytes, n, S, C, monkeypatch):
    """Exact p2p rounds move m consecutive chunks per step (>= the unit
    bytes, fixed by the geometry): same sums and traffic, fewer groups."""
    monkeypatch.setenv("AKKA_EXACT_UNIT_BYTES", unit_bytes)
    cl = SimCluster(n, S, C, max_lag=1, lane="p2p")
    before = 0
    for r in range(3):
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        assert all(torch.equal(o.data, want) and bool((o.count == n).all()) for o in outs)
        assert cl.bytes_moved() - before == 2 * (n - 1) * S * 4
        before = cl.bytes_moved()
    g = Geometry(S, n, C)
    m = max(1, min(-(-int(unit_bytes) // (C * 4)), g.kmax)) if int(unit_bytes) else 1
    st = cl.workers[0].state()["link"]
    assert st["exact_unit_chunks"] == m
    kx, lag = Geometry(S, n, C * m).kmax, 2
    busy = len({s for s in range(kx)} | {s for s in range(lag, kx + lag)})  # steps with any op
    assert st["groups"] == 3 * busy


def test_exact_unit_switch_between_rounds():
    """set_exact_unit_bytes rebuilds the exact template at the next round
    (what bench.py's lane selection does between its candidates): sums stay
    exact and the unit follows the setting, per chunk / whole block / default."""
    n, S, C = 3, 3000, 50
    cl = SimCluster(n, S, C, max_lag=1, lane="p2p")
    g = Geometry(S, n, C)
    for r, (unit, m) in enumerate([(0, 1), (1 << 40, g.kmax), (C * 4 * 3, 3), (0, 1), (-1, None)]):
        for w in cl.workers:
            w.set_exact_unit_bytes(unit)
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        assert all(torch.equal(o.data, want) and bool((o.count == n).all()) for o in outs), (r, unit)
        got = cl.workers[0].state()["link"]["exact_unit_chunks"]
        if m is not None:
            assert got == m, (unit, got)


def test_ipc_lane_needs_open_windows():
    """set_lane('ipc') before the windows are mapped fails loudly (the ipc
    lane itself runs on GPUs only: tests/test_ipc_gpu.py)."""
    cl = SimCluster(2, 100, 10)
    with pytest.raises(Exception, match="ipc"):
        cl.workers[0].set_lane("ipc")
    with pytest.raises(Exception, match="ipc"):
        cl.workers[0].ipc_handle()  # host device: no HIP windows


def test_ipc_data_plane_validation():
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    with pytest.raises(ValueError, match="cuda"):
        ThresholdAllreduce(16, rank=0, world_size=1, device=torch.device("cpu"), data_plane="ipc")
    with pytest.raises(ValueError, match="exact"):
        ThresholdAllreduce(16, rank=0, world_size=1, device=torch.device("cpu"), data_plane="ipc", th_reduce=0.5)
