"""GPU data path at N = 2..8 on one MI355X: every rank has its own HIP
streams, data plane (gfx950 reduce kernels, counts) and StreamLink; ranks
exchange through device copies ordered by the same events RCCL would be
ordered by.  Exact sums/counts over several rounds (ring reuse), uneven
geometry, bf16, thresholds, async hand-off."""
import pytest
import torch

from akka_allreduce_amd.data import Geometry
from akka_allreduce_amd.parallel.loopback import LoopbackCluster

pytestmark = pytest.mark.gpu


def _inputs(n, S, r, dtype=torch.float32):
    g = torch.Generator().manual_seed(100 * r + n)
    return [torch.randint(-8, 9, (S,), generator=g).to(dtype).cuda() for _ in range(n)]


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("S,C", [(1 << 16, 1 << 12), (100_003, 777), (5, 1), ((1 << 20) + 3, 1 << 16)])
def test_loopback_exact(n, S, C):
    cl = LoopbackCluster(n, S, C, max_lag=1)
    for r in range(4):
        xs = _inputs(n, S, r)
        outs = cl.allreduce(xs)
        want = torch.stack(xs).sum(0)
        for rank, o in enumerate(outs):
            torch.cuda.synchronize()
            assert torch.equal(o.data, want), (n, S, C, r, rank)
            assert bool((o.count == n).all()), (n, S, C, r, rank)


def test_loopback_bf16_and_lag():
    n, S, C = 4, 300_001, 4096
    for lag in (1, 2, 3):
        cl = LoopbackCluster(n, S, C, dtype=torch.bfloat16, broadcast_lag=lag)
        xs = _inputs(n, S, lag, torch.bfloat16)
        outs = cl.allreduce(xs)
        want = torch.stack([x.float() for x in xs]).sum(0).bfloat16()
        torch.cuda.synchronize()
        assert all(torch.equal(o.data, want) for o in outs), lag


def test_loopback_async_rounds():
    n, S, C = 4, 1 << 18, 1 << 14
    cl = LoopbackCluster(n, S, C, max_lag=2)
    rounds = [_inputs(n, S, r) for r in range(5)]
    outs = [cl.allreduce(xs, async_op=True) for xs in rounds]
    for xs, os_ in zip(rounds, outs):
        want = torch.stack(xs).sum(0)
        for o in os_:
            o.wait()
            assert torch.equal(o.data, want)


def test_loopback_threshold_subset():
    n, S, C = 4, 4000, 100
    cl = LoopbackCluster(n, S, C, th_reduce=0.75)
    xs = _inputs(n, S, 0)
    outs = cl.allreduce(xs)
    g = Geometry(S, n, C)
    want = torch.zeros(S, device="cuda")
    for j in range(n):
        s, e = g.block_range(j)
        want[s:e] = torch.stack([xs[(j + i) % n][s:e] for i in range(3)]).sum(0)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o.data, want)
        assert bool((o.count == 3).all())


def test_loopback_completion_before_late_chunks():
    """Same as the simulator case: thComplete < 1 completes the round before
    later chunks' broadcast steps; they go out as zeros with count 0."""
    n, S, C, th = 3, 63 * 1024, 1024, 0.67
    cl = LoopbackCluster(n, S, C, th_reduce=th, th_complete=th)
    for _ in range(2):
        outs = cl.allreduce([torch.full((S,), float(1 << i), device="cuda") for i in range(n)])
        torch.cuda.synchronize()
        for o in outs:
            m = o.data.round().long()
            pc = sum(((m >> b) & 1) for b in range(n))
            assert torch.equal(pc.int(), o.count)


def test_loopback_n8_64mib_async():
    """Headline-like shape at N=8 on one GPU: 64 MiB fp32, 4 MiB chunks,
    async back-to-back rounds into one reused output buffer per rank."""
    n, S, C = 8, (64 << 20) // 4, (4 << 20) // 4
    cl = LoopbackCluster(n, S, C, max_lag=2)
    for r in range(3):
        xs = [torch.full((S,), float(r * 10 + i), device="cuda") for i in range(n)]
        outs = cl.allreduce(xs, async_op=True)
        want = float(sum(r * 10 + i for i in range(n)))
        for o in outs:
            o.wait()
        torch.cuda.synchronize()
        for o in outs:
            assert bool((o.data == want).all()) and bool((o.count == n).all())


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("S,C", [(1 << 16, 1 << 12), (100_003, 777), (5, 1)])
def test_loopback_collective_lane(n, S, C):
    """Exact rounds on the whole-round lane with real HIP streams: whole-block
    direct exchange (the loopback endpoint has no native collectives) around
    one gfx950 N-way reduce, several rounds through the ring, async hand-off."""
    cl = LoopbackCluster(n, S, C, max_lag=1, lane="collective")
    rounds = [_inputs(n, S, r) for r in range(4)]
    outs = [cl.allreduce(xs, async_op=True) for xs in rounds]
    for xs, os_ in zip(rounds, outs):
        want = torch.stack(xs).sum(0)
        for o in os_:
            o.wait()
            assert torch.equal(o.data, want)
            assert bool((o.count == n).all())
    st = cl.workers[0].state()
    assert st["link"]["bulk_rounds"] == 4 and st["stats"]["bulk_rounds"] == 4
