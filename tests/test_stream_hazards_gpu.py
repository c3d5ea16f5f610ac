"""Stream-order hazards between the caller's stream and the engine's streams.

The caching allocator hands a round's output/counts memory to the engine in
the caller's stream order: a block freed by the caller may still be written by
work queued earlier on that stream.  Every engine stream that writes the
output or the counts must therefore wait for the point where the caller's
stream handed them over.  Here a pending caller-stream kernel (a spin, then a
fill of -7) owns the block the round's counts table is allocated from; the
round's per-chunk counts must still read N (exact round, all N contributors).

Uses the 1-GPU RCCL shape transport (rank 0 of N, every op to itself), whose
exact rounds run the same engine / data-plane / stream code as N real ranks.
"""
import pytest
import torch

from akka_allreduce_amd import AllreduceWorker, InitWorkers
from akka_allreduce_amd.parallel.collective import _RemoteRank

pytestmark = pytest.mark.gpu


def _shape_worker(n, S, C, sink=None):
    dev = torch.device("cuda", 0)
    w = AllreduceWorker(None, sink, device=dev, transport="stream", transport_spec=("rccl_shape", 0, n),
                        broadcast_lag=2, strict=True, name=f"hazard{n}")
    peers = {i: (w if i == 0 else _RemoteRank(i)) for i in range(n)}
    w.tell(InitWorkers(peers, n, None, 0, 1.0, 1.0, 2, S, C))
    w.set_lane("p2p")
    return w


def _poison_then_free(nbytes):
    """Queue a long spin and then a -7 fill of a fresh block on the current
    stream, free the block (reusable at once in this stream's order), return
    its address range.  On a stream that never allocated before, the round's
    output and then its counts are carved from this block."""
    junk = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
    torch.cuda._sleep(200_000_000)  # ~0.1 s of GPU time before the fill
    junk.fill_(-7)
    lo = junk.data_ptr()
    del junk
    return lo, lo + nbytes


@pytest.mark.parametrize("path", ["fast", "sink"])
def test_counts_written_after_callers_pending_work(path):
    n, S, C = 4, 1 << 16, 1 << 12
    outs = []
    w = _shape_worker(n, S, C, sink=outs.append if path == "sink" else None)
    g = w.geometry
    x = torch.randn(S, device="cuda")
    for _ in range(2):  # warm the allocator and the schedule
        o = w.allreduce(x)
    torch.cuda.synchronize()
    outs.clear()
    side = torch.cuda.Stream()  # its own allocator pool: only the poisoned block is free there
    with torch.cuda.stream(side):
        lo, hi = _poison_then_free(S * 4 + 4096)
        o = w.allreduce(x)
        if path == "sink":
            o = outs[-1]
        pc = o.counts_per_chunk
        # the hazard is only exercised if the counts really sit in the poisoned block
        assert lo <= pc.data_ptr() < hi
    side.synchronize()
    torch.cuda.synchronize()
    assert int(pc.min()) == n and int(pc.max()) == n, pc


@pytest.mark.parametrize("busy", [True, False])
def test_async_round_input_hand_over(busy):
    """An async round on the engine's streams reads the caller's input only
    after the caller's stream produced it.  Busy caller stream (a spin, then
    the kernel that writes the input): the hand-over event must be kept.
    Idle caller stream (everything synchronised): the engine skips that
    event (DataPlane::bind_input, Device::stream_idle) and the round is still
    the exact sum."""
    n, S, C = 4, 1 << 16, 1 << 12
    w = _shape_worker(n, S, C)
    x = torch.ones(S, device="cuda")  # (constant: the shape transport sends every op to itself)
    for _ in range(2):
        w.allreduce(x, async_op=True).wait()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        y = torch.full((S,), -1.0, device="cuda")
        if busy:
            torch.cuda._sleep(200_000_000)  # ~0.1 s of GPU time before the input's final value
            y.fill_(3.0)
        else:
            y.fill_(3.0)
            side.synchronize()
        o = w.allreduce(y, async_op=True)
        o.wait()
        got = o.data.clone()
    side.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(got, torch.full_like(got, 3.0 * n)), (got.min(), got.max())
