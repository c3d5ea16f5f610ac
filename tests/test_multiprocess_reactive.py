"""The reactive (straggler-tolerant) transport across real processes on CPU:
one process per rank, gloo async isend/irecv per pair group (posted from the
pair stream's queue, completion polled), the native ReactiveLink/engine/data
plane unchanged.  Exact sums at thresholds 1; with thresholds < 1 a sleeping
rank does not hold the others back (the reference's core promise), and
every output satisfies the contributor-mask == count invariant."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _w(S):
    return (torch.arange(S) % 3 + 1).float()


def _rank_main(rank, world, port, S, C, th, rounds, sleep_rank, sleep_s, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from akka_allreduce_amd.parallel import ThresholdAllreduce

        ar = ThresholdAllreduce(S, max_chunk_size=C, rank=rank, world_size=world, device=torch.device("cpu"),
                                th_reduce=th, th_complete=th, max_lag=2, transport="reactive")
        ar.worker.reactive_timeout = 60.0
        masks, counts = [], []
        t0 = time.monotonic()
        for r in range(rounds):
            if rank == sleep_rank:
                time.sleep(sleep_s)
            out = ar(_w(S) * float(1 << rank))
            m = (out.data / _w(S)).round().long()
            ok = torch.equal(m.float() * _w(S), out.data)
            pc = sum(((m >> b) & 1) for b in range(world))
            masks.append(m.unique().tolist())
            counts.append(bool(ok) and torch.equal(pc.int(), out.count))
        elapsed = time.monotonic() - t0
        ar.drain(60.0)
        st = ar.state()
        q.put((rank, all(counts), masks, elapsed, st["link"]["in_flight"], st["round"]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e), 0.0, -1, -1))


def _run(world, S, C, th, rounds, sleep_rank=-1, sleep_s=0.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, S, C, th, rounds, sleep_rank, sleep_s, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,S,C", [(2, 1000, 64), (3, 777, 50), (4, 4099, 128)])
def test_reactive_multiprocess_exact(world, S, C):
    res = _run(world, S, C, 1.0, 4)
    full = (1 << world) - 1
    for rank, ok, masks, _, inflight, rnd in res:
        assert ok, (rank, masks)
        assert all(m == [full] for m in masks), (rank, masks)
        assert inflight == 0 and rnd == 4


def test_reactive_multiprocess_sleeping_rank():
    """Rank 2 of 3 sleeps 0.5 s before every round; at th = 0.67 ranks 0 and 1
    complete all rounds from each other's data without waiting for it."""
    world, S, C, R, nap = 3, 3000, 100, 4, 0.5
    res = _run(world, S, C, 0.67, R, sleep_rank=2, sleep_s=nap)
    for rank, ok, masks, elapsed, inflight, rnd in res:
        assert ok, (rank, masks)
        assert inflight == 0 and rnd == R
        if rank < 2:
            assert elapsed < nap * R / 2, (rank, elapsed)  # never waited for the sleeper
            g = masks  # blocks 0 and 1 reduced from {0, 1}; block 2 never reduced (0)
            assert all(set(m) <= {0, 0b011} for m in g), (rank, masks)
