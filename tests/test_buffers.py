"""Buffer semantics (reference ScatteredDataBufferSpec / ReducedDataBufferSpec,
B1-B7 in SURVEY §4.1), asserted through the native engine + data plane that
replace AllReduceBuffer/ScatteredDataBuffer/ReducedDataBuffer.

The reference tests the buffer classes directly; here the same properties
are observed through a worker driven by messages (the buffers are internal
to the engine), plus the geometry/threshold helpers the buffers derive from.
"""
import pytest
import torch

from akka_allreduce_amd import AllreduceWorker
from akka_allreduce_amd.data import Geometry
from akka_allreduce_amd.messages import CompleteAllreduce, InitWorkers, ReduceBlock, ScatterBlock, StartAllreduce
from akka_allreduce_amd.testing import TestProbe, initialize_workers_as


def _worker(n, S, C, thR, thC, lag, idx=0, sink=None, src=None):
    probe = TestProbe()
    w = AllreduceWorker(src or (lambda req: torch.zeros(S)), sink, strict=True)
    w.tell(InitWorkers(initialize_workers_as(probe, n), n, probe, idx, thR, thC, lag, S, C))
    return w, probe


# B1 -- "initialize buffers": maxLag rows x peers x block (SBS:24-30, RBS:24-30)
def test_b1_dimensions():
    w, _ = _worker(4, 20, 3, 0.75, 1.0, 3)
    st = w.state()
    assert st["ring_rows"] == 4           # maxLag + 1 rows (W:64)
    g = Geometry(20, 4, 3)
    assert [g.block_len(j) for j in range(4)] == [5, 5, 5, 5]
    assert [g.num_chunks(j) for j in range(4)] == [2, 2, 2, 2]
    assert st["kmax"] == 2


# B2 -- "throw when store exceeds expected size" (SBS:32-42, RBS:54-70)
def test_b2_store_overrun_raises_short_last_chunk_ok():
    # block 5, chunk 3 -> chunks of 3 and 2; a full 3-element store into the last chunk must fail
    w, probe = _worker(4, 20, 3, 1.0, 1.0, 3)
    w.tell(StartAllreduce(0))
    probe.drain()
    with pytest.raises(RuntimeError, match="overruns"):
        w.tell(ScatterBlock([1.0, 2.0, 3.0], 1, 0, 1, 0))
    w.tell(ScatterBlock([1.0, 2.0], 1, 0, 1, 0))  # short last chunk is fine
    assert w.state()["stats"]["scatters_in"] >= 1
    with pytest.raises(RuntimeError):
        w.tell(ReduceBlock([1.0, 2.0, 3.0, 4.0], 1, 0, 0, 0, 4))  # > maxChunkSize (W:150-151)


# B3 -- "reach reducing threshold": th .75 of 4 -> false, false, true (SBS:44-54)
def test_b3_reducing_threshold_sequence():
    w, probe = _worker(4, 20, 3, 0.75, 1.0, 3)
    w.tell(StartAllreduce(0))
    probe.drain()
    fired = []
    for src in range(3):
        w.tell(ScatterBlock([1.0, 1.0, 1.0], src, 0, 0, 0))
        fired.append(any(isinstance(m, ReduceBlock) for m in probe.drain()))
    assert fired == [False, False, True]
    assert w._core.scatter_count(0, 0) == 3


# B4 -- "reduce values with correct count": empty row -> zeros, count 0 (SBS:56-64)
def test_b4_forced_reduce_of_empty_row():
    w, probe = _worker(4, 8, 2, 1.0, 1.0, 0)  # maxLag 0: StartAllreduce(1) forces round 0
    w.tell(StartAllreduce(0))
    probe.drain()
    w.tell(StartAllreduce(1))
    red = [m for m in probe.drain() if isinstance(m, ReduceBlock) and m.round == 0]
    assert red and all(m.count == 0 and m.value.sum() == 0 for m in red)


# B5 -- "sum from all peers at one row" / "not affected by other rows" (SBS:80-102)
def test_b5_sum_and_row_isolation():
    # block 2, chunk 3 > block: one chunk per block; row 0 and row 1 are independent
    w, probe = _worker(2, 4, 3, 1.0, 1.0, 2)
    w.tell(StartAllreduce(0))
    w.tell(StartAllreduce(1))
    probe.drain()
    for i in range(2):
        w.tell(ScatterBlock([float(i), float(i)], i, 0, 0, 0))
    red0 = [m for m in probe.drain() if isinstance(m, ReduceBlock)]
    assert red0 and red0[0].value.tolist() == [1.0, 1.0] and red0[0].count == 2
    assert w._core.scatter_count(1, 0) == 0  # other row untouched


# B6 -- reduced buffer, even blocks: completion at floor(.7*9)=6, missing chunks
# read as 0 with count 0 (RBS:24-119)
def test_b6_reduced_even_blocks_missing_chunks():
    out = []
    w, probe = _worker(3, 15, 2, 1.0, 0.7, 3, sink=out.append)
    assert w.state()["min_reduced_required"] == 6
    w.tell(StartAllreduce(0))
    probe.drain()
    stores = [(0, 0), (0, 1), (1, 0), (1, 1), (2, 1)]  # peer 2 chunk 1 ... (RBS order, then the 6th)
    for src, k in stores:
        w.tell(ReduceBlock([7.0, 7.0], src, 0, k, 0, 3))
        assert not out
    w.tell(ReduceBlock([7.0], 2, 0, 2, 0, 3))  # 6th chunk (last, short) -> complete
    assert len(out) == 1 and isinstance(probe.drain()[-1], CompleteAllreduce)
    data, count = out[0].data.tolist(), out[0].count.tolist()
    missing = [4, 9, 10, 11]  # same indices as RBS:103 (peers 0,1 lack chunk 2; peer 2 lacks chunk 0)
    for i in range(15):
        if i in missing:
            assert data[i] == 0 and count[i] == 0, i
        else:
            assert data[i] == 7.0 and count[i] == 3, i


# B7 -- reduced buffer, uneven blocks: completion exactly at all 8 chunks (RBS:124-158)
def test_b7_reduced_uneven_blocks_completion():
    g = Geometry(16, 3, 2)
    assert [g.block_len(j) for j in range(3)] == [6, 6, 4]
    assert g.total_chunks == 8
    out = []
    w, probe = _worker(3, 16, 2, 1.0, 1.0, 3, sink=out.append)
    assert w.state()["min_reduced_required"] == 8
    w.tell(StartAllreduce(0))
    for k in range(3):
        for src in range(2):
            w.tell(ReduceBlock([1.0, 1.0], src, 0, k, 0, 3))
            assert not out
    w.tell(ReduceBlock([1.0, 1.0], 2, 0, 0, 0, 3))
    assert not out
    w.tell(ReduceBlock([1.0, 1.0], 2, 0, 1, 0, 3))
    assert len(out) == 1 and bool((out[0].count == 3).all())


# Reference quirk regressions ------------------------------------------------
def test_quirk2_duplicates_neither_overshoot_nor_stall():
    """The reference's `==` thresholds never fire once a duplicate overshoots
    the count; distinct-source counting + fire-once does."""
    w, probe = _worker(4, 4, 2, 0.75, 0.75, 5)
    w.tell(StartAllreduce(0))
    probe.drain()
    w.tell(ScatterBlock([1.0], 1, 0, 0, 0))
    w.tell(ScatterBlock([1.0], 1, 0, 0, 0))  # duplicate: still 1 distinct
    assert not any(isinstance(m, ReduceBlock) for m in probe.drain())
    w.tell(ScatterBlock([1.0], 2, 0, 0, 0))
    w.tell(ScatterBlock([1.0], 3, 0, 0, 0))  # 3 distinct -> reduce
    red = [m for m in probe.drain() if isinstance(m, ReduceBlock)]
    assert len(red) == 4 and red[0].count == 3


def test_quirk34_exact_partitioning_large_and_tiny():
    g = Geometry(16_777_217, 8, 1 << 20)  # float32 ceil misrounds here in the reference
    assert g.step == 2_097_153
    assert sum(g.block_len(j) for j in range(8)) == 16_777_217
    assert max(g.block_len(j) for j in range(8)) == g.step
    g = Geometry(5, 4, 1)  # reference indexes out of bounds (fewer range entries than workers)
    assert [g.block_len(j) for j in range(4)] == [2, 2, 1, 0]
    w, probe = _worker(4, 5, 1, 1.0, 1.0, 1, idx=3)  # worker with an empty block
    w.tell(StartAllreduce(0))
    assert len([m for m in probe.drain() if isinstance(m, ScatterBlock)]) == 5


def test_quirk1_catchup_never_double_completes():
    """Self-delivery during a forced round completes it; the catch-up loop must
    not then force-complete the next round by accident (W:100-106)."""
    out = []
    probe = TestProbe()
    w = AllreduceWorker(lambda req: torch.ones(2), out.append, strict=True)
    workers = {0: w, 1: probe}
    # thComplete 0.5 of 2 chunks: my own self-delivered reduced chunk completes the round
    w.tell(InitWorkers(workers, 2, probe, 0, 1.0, 0.5, 0, 2, 1))
    w.tell(StartAllreduce(0))
    w.tell(StartAllreduce(3))  # force rounds 0..2
    rounds = [m.round for m in probe.drain() if isinstance(m, CompleteAllreduce)]
    assert rounds == sorted(set(rounds)) == [0, 1, 2]
    assert [o.iteration for o in out] == [0, 1, 2]
