"""Behavioural spec of the worker: one test per case of the reference's
AllReduceSpec (src/test/scala/AllreduceSpec.scala), T1-T18 in SURVEY §4.1.

As in the reference, one real worker runs and every peer and the master is a
probe, so the test plays the other workers and sees every outgoing message in
order.  Each case runs on the host data plane (CPU) and, marked ``gpu``, on
the HIP data plane where every chunk sum is the gfx950 reduce kernel.
Deviations from the reference are deliberate quirk fixes and
are called out where they change an expectation (none of T1-T18 changes).
"""
import pytest
import torch

from akka_allreduce_amd import AllreduceWorker
from akka_allreduce_amd.messages import CompleteAllreduce, InitWorkers, ReduceBlock, ScatterBlock, StartAllreduce
from akka_allreduce_amd.testing import (
    TestProbe,
    assertive_data_sink,
    create_basic_data_source,
    create_custom_data_source,
    initialize_workers_as,
)

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def printing_sink(r):
    pass


def make(source, sink, device, **kw):
    return AllreduceWorker(source, sink, device=device, strict=True, **kw)


@pytest.fixture
def probe():
    return TestProbe()


# SPEC:46-97 (T1) -----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t1_sum_up_all_correct_data(probe, device):
    idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize, workerNum = 1, 1.0, 1.0, 5, 3, 2, 2
    gen = lambda i, it: float(i + it)
    source = create_custom_data_source(dataSize, gen)
    out1 = [gen(i, 0) * workerNum for i in range(dataSize)]
    out2 = [gen(i, 1) * workerNum for i in range(dataSize)]
    seen = []
    sink = assertive_data_sink([out1, out2], [[2, 2, 2], [2, 2, 2]], [0, 1], seen)
    worker = make(source, sink, device)
    # self mapped to the real worker: it delivers to itself directly (SPEC:74-75)
    workers = initialize_workers_as(probe, workerNum)
    workers[idx] = worker
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize))
    worker.tell(StartAllreduce(0))
    worker.tell(ScatterBlock([2.0], srcId=0, destId=1, chunkId=0, round=0))
    worker.tell(ReduceBlock([0.0, 2.0], srcId=0, destId=1, chunkId=0, round=0, count=2))
    worker.tell(StartAllreduce(1))
    worker.tell(ScatterBlock([3.0], srcId=0, destId=1, chunkId=0, round=1))
    worker.tell(ReduceBlock([2.0, 4.0], srcId=0, destId=1, chunkId=0, round=1, count=2))
    probe.fish_for_message(lambda m: m == CompleteAllreduce(1, 0))
    probe.fish_for_message(lambda m: m == CompleteAllreduce(1, 1))
    assert seen == [0, 1]


# SPEC:99-139 (T2, T3) ---------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t2_t3_early_receiving_reduce(probe, device):
    idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize, workerNum = 0, 1.0, 0.8, 5, 8, 2, 4
    worker = make(create_basic_data_source(8), printing_sink, device)
    workers = initialize_workers_as(probe, workerNum)
    future = 3
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize))
    worker.tell(StartAllreduce(0))
    worker.tell(ReduceBlock([12.0, 15.0], 0, 0, 0, future, count=4))
    worker.tell(ReduceBlock([11.0, 10.0], 1, 0, 0, future, count=4))
    worker.tell(ReduceBlock([10.0, 20.0], 2, 0, 0, future, count=4))
    worker.tell(ReduceBlock([9.0, 10.0], 3, 0, 0, future, count=4))

    def pred(m):
        if isinstance(m, CompleteAllreduce):
            assert m.round == future and m.srcId == 0
            return True
        assert isinstance(m, ScatterBlock)
        return False

    probe.fish_for_message(pred)
    # T3: no longer act on completed scatter for that round
    probe.drain()
    for i in range(4):
        worker.tell(ScatterBlock([2.0 * i, 2.0 * i], srcId=i, destId=0, chunkId=0, round=future))
    probe.expect_no_msg()


# SPEC:141-172 (T4, T5) --------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t4_t5_nodes_live_at_different_times(probe, device):
    idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize, workerNum = 0, 1.0, 1.0, 5, 8, 2, 4
    worker = make(create_basic_data_source(8), printing_sink, device)
    workers = initialize_workers_as(probe, workerNum)
    incomplete = {0: workers[0]}
    # T4: only send one scatter
    worker.tell(InitWorkers(incomplete, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize))
    worker.tell(StartAllreduce(0))
    probe.expect_scatter([0.0, 1.0], srcId=0, destId=0, chunkId=0, round=0)
    probe.expect_no_msg()
    # T5: send all scatters after all peers joined
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxMsgSize))
    worker.tell(StartAllreduce(1))
    for i in range(4):
        probe.expect_scatter([2.0 * i + 1, 2.0 * i + 2], srcId=0, destId=i, chunkId=0, round=1)


# SPEC:175-213 (T6) -----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t6_single_round_allreduce(probe, device):
    worker = make(create_basic_data_source(8), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 4, 0, 1.0, 0.75, 5, 8, 2
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    for i in range(4):
        probe.expect_scatter([2.0 * i, 2.0 * i + 1], 0, i, 0, 0)
    for i in range(4):
        worker.tell(ScatterBlock([2.0 * i, 2.0 * i], i, 0, 0, 0))
    for d in range(4):
        probe.expect_reduce([12.0, 12.0], 0, d, 0, 0, 4)
    worker.tell(ReduceBlock([12.0, 15.0], 0, 0, 0, 0, 4))
    worker.tell(ReduceBlock([11.0, 10.0], 1, 0, 0, 0, 4))
    worker.tell(ReduceBlock([10.0, 20.0], 2, 0, 0, 0, 4))
    worker.tell(ReduceBlock([9.0, 10.0], 3, 0, 0, 0, 4))
    probe.expect_msg(CompleteAllreduce(0, 0))


# SPEC:215-238 (T7) -----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t7_uneven_size_sending_to_self_first(probe, device):
    dataSize = 3
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, maxChunkSize = 2, 1, 1.0, 1.0, 1, 1
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    probe.expect_scatter([2.0], srcId=1, destId=1, chunkId=0, round=0)
    probe.expect_scatter([0.0], srcId=1, destId=0, chunkId=0, round=0)
    probe.expect_scatter([1.0], srcId=1, destId=0, chunkId=1, round=0)


# SPEC:240-284 (T8) -----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t8_nasty_chunk_size(probe, device):
    dataSize = 6
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, maxChunkSize = 2, 0, 0.9, 0.8, 5, 2
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    probe.expect_scatter([0.0, 1.0], 0, 0, 0, 0)
    probe.expect_scatter([2.0], 0, 0, 1, 0)
    probe.expect_scatter([3.0, 4.0], 0, 1, 0, 0)
    probe.expect_scatter([5.0], 0, 1, 1, 0)
    worker.tell(ScatterBlock([0.0, 1.0], 0, 0, 0, 0))
    worker.tell(ScatterBlock([2.0], 0, 0, 1, 0))
    worker.tell(ScatterBlock([0.0, 1.0], 1, 0, 0, 0))
    worker.tell(ScatterBlock([2.0], 1, 0, 1, 0))
    probe.expect_reduce([0.0, 1.0], 0, 0, 0, 0, 1)
    probe.expect_reduce([0.0, 1.0], 0, 1, 0, 0, 1)
    probe.expect_reduce([2.0], 0, 0, 1, 0, 1)
    probe.expect_reduce([2.0], 0, 1, 1, 0, 1)
    worker.tell(ReduceBlock([0.0, 2.0], 0, 0, 0, 0, 1))
    worker.tell(ReduceBlock([4.0], 0, 0, 1, 0, 1))
    worker.tell(ReduceBlock([6.0, 8.0], 1, 0, 0, 0, 1))
    probe.expect_msg(CompleteAllreduce(0, 0))
    worker.tell(ReduceBlock([10.0], 1, 0, 1, 0, 1))
    probe.expect_no_msg()


# SPEC:286-349 (T9) -----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t9_nasty_chunk_size_contd(probe, device):
    dataSize = 9
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, maxChunkSize = 3, 0, 0.7, 0.7, 5, 1
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    for dest in range(3):
        for k in range(3):
            probe.expect_scatter([float(3 * dest + k)], 0, dest, k, 0)
    for src in range(3):
        for k in range(3):
            worker.tell(ScatterBlock([float(k)], src, 0, k, 0))
    for k in range(3):
        for d in range(3):
            probe.expect_reduce([float(2 * k)], 0, d, k, 0, 2)
    worker.tell(ReduceBlock([0.0], 0, 0, 0, 0, 2))
    worker.tell(ReduceBlock([3.0], 0, 0, 1, 0, 2))
    worker.tell(ReduceBlock([6.0], 0, 0, 2, 0, 2))
    worker.tell(ReduceBlock([9.0], 1, 0, 0, 0, 2))
    worker.tell(ReduceBlock([12.0], 1, 0, 1, 0, 2))
    worker.tell(ReduceBlock([15.0], 1, 0, 2, 0, 2))
    worker.tell(ReduceBlock([18.0], 2, 0, 0, 0, 2))
    probe.expect_msg(CompleteAllreduce(0, 0))
    worker.tell(ReduceBlock([21.0], 2, 0, 1, 0, 2))
    worker.tell(ReduceBlock([24.0], 2, 0, 2, 0, 2))
    probe.expect_no_msg()


# SPEC:351-385 (T10) ----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t10_multi_round_allreduce(probe, device):
    worker = make(create_basic_data_source(8), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 4, 0, 0.8, 0.5, 5, 8, 2
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    for i in range(10):
        worker.tell(StartAllreduce(i))
        probe.expect_scatter([0.0 + i, 1.0 + i], 0, 0, 0, i)
        probe.expect_scatter([2.0 + i, 3.0 + i], 0, 1, 0, i)
        probe.expect_scatter([4.0 + i, 5.0 + i], 0, 2, 0, i)
        probe.expect_scatter([6.0 + i, 7.0 + i], 0, 3, 0, i)
        for s in range(4):
            worker.tell(ScatterBlock([0.0 + i, 1.0 + i], s, 0, 0, i))
        for d in range(4):
            probe.expect_reduce([0.0 + 3 * i, 3.0 + 3 * i], 0, d, 0, i, 3)
        worker.tell(ReduceBlock([1.0, 2.0], 0, 0, 0, i, 3))
        worker.tell(ReduceBlock([1.0, 2.0], 1, 0, 0, i, 3))
        probe.expect_msg(CompleteAllreduce(0, i))
        worker.tell(ReduceBlock([1.0, 2.0], 2, 0, 0, i, 3))
        worker.tell(ReduceBlock([1.0, 2.0], 3, 0, 0, i, 3))
        probe.expect_no_msg()


# SPEC:387-422 (T11) ----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t11_multi_round_allreduce_v2(probe, device):
    worker = make(create_basic_data_source(8), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 2, 0, 0.6, 0.8, 5, 8, 2
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    for i in range(10):
        worker.tell(StartAllreduce(i))
        probe.expect_scatter([0.0 + i, 1.0 + i], 0, 0, 0, i)
        probe.expect_scatter([2.0 + i, 3.0 + i], 0, 0, 1, i)
        probe.expect_scatter([4.0 + i, 5.0 + i], 0, 1, 0, i)
        probe.expect_scatter([6.0 + i, 7.0 + i], 0, 1, 1, i)
        worker.tell(ScatterBlock([0.0 + i, 1.0 + i], 0, 0, 0, i))
        worker.tell(ScatterBlock([2.0 + i, 3.0 + i], 0, 0, 1, i))
        worker.tell(ScatterBlock([10.0 + i, 11.0 + i], 1, 0, 0, i))
        worker.tell(ScatterBlock([12.0 + i, 13.0 + i], 1, 0, 1, i))
        probe.expect_reduce([0.0 + i, 1.0 + i], 0, 0, 0, i, 1)
        probe.expect_reduce([0.0 + i, 1.0 + i], 0, 1, 0, i, 1)
        probe.expect_reduce([2.0 + i, 3.0 + i], 0, 0, 1, i, 1)
        probe.expect_reduce([2.0 + i, 3.0 + i], 0, 1, 1, i, 1)
        worker.tell(ReduceBlock([1.0, 2.0], 0, 0, 0, i, 1))
        worker.tell(ReduceBlock([1.0, 2.0], 0, 0, 1, i, 1))
        worker.tell(ReduceBlock([1.0, 2.0], 1, 0, 0, i, 1))
        probe.expect_msg(CompleteAllreduce(0, i))
        worker.tell(ReduceBlock([1.0, 2.0], 1, 0, 1, i, 1))
        probe.expect_no_msg()


# SPEC:424-459 (T12) ----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t12_missed_scatter(probe, device):
    workerNum, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 4, 0, 0.75, 0.75, 5, 4, 2
    workers = initialize_workers_as(probe, workerNum)
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    for d in range(4):
        probe.expect_scatter([float(d)], 0, d, 0, 0)
    worker.tell(ScatterBlock([0.0], 0, 0, 0, 0))
    probe.expect_no_msg()
    worker.tell(ScatterBlock([2.0], 1, 0, 0, 0))
    probe.expect_no_msg()
    worker.tell(ScatterBlock([4.0], 2, 0, 0, 0))
    worker.tell(ScatterBlock([6.0], 3, 0, 0, 0))
    for d in range(4):
        probe.expect_reduce([6.0], 0, d, 0, 0, 3)
    worker.tell(ReduceBlock([12.0], 0, 0, 0, 0, 3))
    worker.tell(ReduceBlock([11.0], 1, 0, 0, 0, 3))
    worker.tell(ReduceBlock([10.0], 2, 0, 0, 0, 3))
    probe.expect_msg(CompleteAllreduce(0, 0))
    worker.tell(ReduceBlock([9.0], 3, 0, 0, 0, 3))
    probe.expect_no_msg()


# SPEC:461-513 (T13) ----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t13_future_scatter(probe, device):
    workerNum, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 4, 0, 0.75, 0.75, 5, 4, 2
    workers = initialize_workers_as(probe, workerNum)
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    for d in range(4):
        probe.expect_scatter([float(d)], 0, d, 0, 0)
    worker.tell(ScatterBlock([2.0], 1, 0, 0, 0))
    worker.tell(ScatterBlock([4.0], 2, 0, 0, 0))
    worker.tell(ReduceBlock([11.0], 1, 0, 0, 0, 3))
    worker.tell(ReduceBlock([10.0], 2, 0, 0, 0, 3))
    # two of the messages are delayed, so now stall
    worker.tell(StartAllreduce(1))
    worker.tell(ScatterBlock([2.0], 1, 0, 0, 1))
    worker.tell(ScatterBlock([4.0], 2, 0, 0, 1))
    worker.tell(ScatterBlock([6.0], 3, 0, 0, 1))
    for d in range(4):
        probe.expect_scatter([1.0 + d], 0, d, 0, 1)
    for d in range(4):
        probe.expect_reduce([12.0], 0, d, 0, 1, 3)
    # delayed message now gets there
    worker.tell(ScatterBlock([0.0], 3, 0, 0, 0))
    worker.tell(ScatterBlock([6.0], 3, 0, 0, 0))  # duplicate: must not re-reduce
    for d in range(4):
        probe.expect_reduce([6.0], 0, d, 0, 0, 3)
    worker.tell(ReduceBlock([9.0], 3, 0, 0, 0, 3))
    probe.expect_msg(CompleteAllreduce(0, 0))
    worker.tell(ReduceBlock([11.0], 1, 0, 0, 1, 3))
    worker.tell(ReduceBlock([10.0], 2, 0, 0, 1, 3))
    worker.tell(ReduceBlock([9.0], 3, 0, 0, 1, 3))
    probe.expect_msg(CompleteAllreduce(0, 1))


# SPEC:515-548 (T14) ----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t14_missed_reduce(probe, device):
    workerNum, idx, thReduce, thComplete, dataSize, maxChunkSize, maxLag = 4, 0, 1.0, 0.75, 4, 100, 5
    workers = initialize_workers_as(probe, workerNum)
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    for d in range(4):
        probe.expect_scatter([float(d)], 0, d, 0, 0)
    for s in range(4):
        worker.tell(ScatterBlock([2.0 * s], s, 0, 0, 0))
    for d in range(4):
        probe.expect_reduce([12.0], 0, d, 0, 0, 4)
    worker.tell(ReduceBlock([12.0], 0, 0, 0, 0, 4))
    probe.expect_no_msg()
    worker.tell(ReduceBlock([11.0], 1, 0, 0, 0, 4))
    probe.expect_no_msg()
    worker.tell(ReduceBlock([10.0], 2, 0, 0, 0, 4))
    probe.expect_msg(CompleteAllreduce(0, 0))


# SPEC:550-599 (T15) ----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t15_delayed_future_reduce(probe, device):
    workerNum, idx, thReduce, thComplete, dataSize, maxChunkSize, maxLag = 4, 0, 0.75, 0.75, 4, 100, 5
    workers = initialize_workers_as(probe, workerNum)
    worker = make(create_basic_data_source(4), printing_sink, device)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    for d in range(4):
        probe.expect_scatter([float(d)], 0, d, 0, 0)
    worker.tell(ScatterBlock([2.0], 1, 0, 0, 0))
    worker.tell(ScatterBlock([4.0], 2, 0, 0, 0))
    worker.tell(ScatterBlock([6.0], 3, 0, 0, 0))
    for d in range(4):
        probe.expect_reduce([12.0], 0, d, 0, 0, 3)
    worker.tell(StartAllreduce(1))
    worker.tell(ScatterBlock([3.0], 1, 0, 0, 1))
    worker.tell(ScatterBlock([5.0], 2, 0, 0, 1))
    worker.tell(ScatterBlock([7.0], 3, 0, 0, 1))
    for d in range(4):
        probe.expect_scatter([1.0 + d], 0, d, 0, 1)
    for d in range(4):
        probe.expect_reduce([15.0], 0, d, 0, 1, 3)
    # reduce t never comes after reduce t+1 from one peer (per-pair FIFO, SPEC:590)
    worker.tell(ReduceBlock([11.0], 1, 0, 0, 0, 3))
    worker.tell(ReduceBlock([11.0], 1, 0, 0, 1, 3))
    worker.tell(ReduceBlock([10.0], 2, 0, 0, 0, 3))
    worker.tell(ReduceBlock([10.0], 2, 0, 0, 1, 3))
    worker.tell(ReduceBlock([9.0], 3, 0, 0, 0, 3))
    worker.tell(ReduceBlock([9.0], 3, 0, 0, 1, 3))
    probe.expect_msg(CompleteAllreduce(0, 0))
    probe.expect_msg(CompleteAllreduce(0, 1))


# SPEC:603-656 (T16, T17) ---------------------------------------------------------------
def _expect_basic_scatter(probe, i):
    probe.expect_scatter([0.0 + i, 1.0 + i], 0, 0, 0, i)
    probe.expect_scatter([2.0 + i, 3.0 + i], 0, 1, 0, i)
    probe.expect_scatter([4.0 + i, 5.0 + i], 0, 2, 0, i)
    probe.expect_scatter([6.0 + i, 7.0 + i], 0, 3, 0, i)


def _simulate_peer_scatters(worker, i):
    worker.tell(ScatterBlock([1.0 * (i + 1)] * 2, 1, 0, 0, i))
    worker.tell(ScatterBlock([2.0 * (i + 1)] * 2, 2, 0, 0, i))
    worker.tell(ScatterBlock([4.0 * (i + 1)] * 2, 3, 0, 0, i))


def _test_catchup(worker, probe, maxLag, catchup_round):
    worker.tell(StartAllreduce(catchup_round))
    completion = catchup_round - (maxLag + 1)
    for d in range(4):
        probe.expect_reduce([7.0 * (completion + 1)] * 2, 0, d, 0, completion, 3)
    probe.expect_msg(CompleteAllreduce(0, completion))
    _expect_basic_scatter(probe, catchup_round)


@pytest.mark.parametrize("device", DEVICES)
def test_t16_simple_catchup(probe, device):
    worker = make(create_basic_data_source(8), printing_sink, device)
    workerNum, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 4, 0, 1.0, 1.0, 5, 8, 2
    workers = initialize_workers_as(probe, workerNum)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    for i in range(6):
        worker.tell(StartAllreduce(i))
        _expect_basic_scatter(probe, i)
        _simulate_peer_scatters(worker, i)
        worker.tell(ReduceBlock([12.0, 12.0], 1, 0, 0, i, 4))
        worker.tell(ReduceBlock([12.0, 12.0], 2, 0, 0, i, 4))
        worker.tell(ReduceBlock([12.0, 12.0], 3, 0, 0, i, 4))
    probe.expect_no_msg()
    _test_catchup(worker, probe, maxLag, 6)
    _test_catchup(worker, probe, maxLag, 7)
    _test_catchup(worker, probe, maxLag, 8)


@pytest.mark.parametrize("device", DEVICES)
def test_t17_cold_catchup(probe, device):
    workerNum = 4
    worker = make(create_basic_data_source(8), printing_sink, device)
    workers = initialize_workers_as(probe, workerNum)
    idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize = 0, 1.0, 1.0, 5, 8, 2
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(10))
    for i in range(5):
        for d in range(4):
            probe.expect_reduce([0.0, 0.0], 0, d, 0, i, 0)
        probe.expect_msg(CompleteAllreduce(0, i))
    # rounds 0..10 are all scattered, including the forced ones (peers may still need them)
    for i in range(11):
        _expect_basic_scatter(probe, i)
    probe.expect_no_msg()


# SPEC:662-734 (T18) -----------------------------------------------------------------
@pytest.mark.parametrize("device", DEVICES)
def test_t18_multi_round_v3_out_of_order_completion(probe, device):
    workerNum, idx, thReduce, thComplete, dataSize, maxChunkSize, maxLag = 3, 0, 0.75, 0.75, 9, 2, 5
    workers = initialize_workers_as(probe, workerNum)
    worker = make(create_basic_data_source(dataSize), printing_sink, device)
    worker.tell(InitWorkers(workers, workerNum, probe, idx, thReduce, thComplete, maxLag, dataSize, maxChunkSize))
    worker.tell(StartAllreduce(0))
    probe.expect_scatter([0.0, 1.0], 0, 0, 0, 0)
    probe.expect_scatter([2.0], 0, 0, 1, 0)
    probe.expect_scatter([3.0, 4.0], 0, 1, 0, 0)
    probe.expect_scatter([5.0], 0, 1, 1, 0)
    probe.expect_scatter([6.0, 7.0], 0, 2, 0, 0)
    probe.expect_scatter([8.0], 0, 2, 1, 0)
    worker.tell(ScatterBlock([0.0, 1.0], 0, 0, 0, 0))
    worker.tell(ScatterBlock([0.0, 1.0], 1, 0, 0, 0))
    worker.tell(ScatterBlock([0.0, 1.0], 2, 0, 0, 0))
    worker.tell(ScatterBlock([2.0], 0, 0, 1, 0))
    worker.tell(ScatterBlock([2.0], 1, 0, 1, 0))
    worker.tell(ScatterBlock([2.0], 2, 0, 1, 0))
    for d in range(3):
        probe.expect_reduce([0.0, 2.0], 0, d, 0, 0, 2)
    for d in range(3):
        probe.expect_reduce([4.0], 0, d, 1, 0, 2)
    worker.tell(StartAllreduce(1))
    worker.tell(ScatterBlock([10.0, 11.0], 1, 0, 0, 1))
    worker.tell(ScatterBlock([12.0], 1, 0, 1, 1))
    worker.tell(ScatterBlock([10.0, 11.0], 2, 0, 0, 1))
    worker.tell(ScatterBlock([12.0], 2, 0, 1, 1))
    probe.expect_scatter([1.0, 2.0], 0, 0, 0, 1)
    probe.expect_scatter([3.0], 0, 0, 1, 1)
    probe.expect_scatter([4.0, 5.0], 0, 1, 0, 1)
    probe.expect_scatter([6.0], 0, 1, 1, 1)
    probe.expect_scatter([7.0, 8.0], 0, 2, 0, 1)
    probe.expect_scatter([9.0], 0, 2, 1, 1)
    for d in range(3):
        probe.expect_reduce([20.0, 22.0], 0, d, 0, 1, 2)
    for d in range(3):
        probe.expect_reduce([24.0], 0, d, 1, 1, 2)
    worker.tell(ReduceBlock([11.0, 11.0], 1, 0, 0, 0, 2))
    worker.tell(ReduceBlock([11.0], 1, 0, 1, 1, 2))
    worker.tell(ReduceBlock([11.0, 11.0], 1, 0, 0, 1, 2))
    worker.tell(ReduceBlock([11.0], 1, 0, 1, 0, 2))
    worker.tell(ReduceBlock([11.0, 11.0], 2, 0, 0, 0, 2))
    worker.tell(ReduceBlock([11.0], 2, 0, 1, 1, 2))
    probe.expect_no_msg()
    worker.tell(ReduceBlock([11.0, 11.0], 2, 0, 0, 1, 2))
    probe.expect_msg(CompleteAllreduce(0, 1))
    worker.tell(ReduceBlock([11.0], 2, 0, 1, 0, 2))
    probe.expect_msg(CompleteAllreduce(0, 0))
    assert worker.round == 2
