"""thAllreduce pacing in the SPMD front end (the reference master's third
straggler knob, M:54-63): round r starts on a rank once thAllreduce*N ranks
completed round r-1 (counters in the job's TCPStore).  Four CPU processes on
the reactive transport (gloo) or the one-sided lane (shared-memory windows),
rank 3 sleeps before every round:
  * thAllreduce = 0.75 -- the pacing advances on ranks 0-2 alone;
  * thAllreduce = 1.0  -- every round waits for the sleeper."""
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


def _rank_main(rank, world, port, th_allreduce, rounds, nap, q, transport="reactive"):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from akka_allreduce_amd.parallel import ThresholdAllreduce

        S = 4096
        ar = ThresholdAllreduce(S, max_chunk_size=256, rank=rank, world_size=world, device=torch.device("cpu"),
                                th_reduce=0.75, th_complete=0.75, max_lag=2, transport=transport,
                                th_allreduce=th_allreduce)
        if transport == "reactive":
            ar.worker.reactive_timeout = 60.0
        t0 = time.monotonic()
        last = -1
        # the job ends at a common ROUND (the master's maxRound, M:58-63): on
        # the one-sided lane the sleeper skips rounds by catch-up
        while last < rounds - 1:
            if rank == world - 1:
                time.sleep(nap)
            o = ar(torch.full((S,), float(rank + 1)))
            last = o.iteration if transport == "onesided" else last + 1
        elapsed = time.monotonic() - t0
        ar.drain(60.0)
        ar.retire()
        dist.barrier()  # every rank passed every round's start
        # pacing keys of rounds everyone passed are gone (only the last round's
        # stays; the one-sided lane's catch-up skips rounds, whose keys stay)
        store = ar.pacer.store
        left = [r for r in range(rounds - 1)
                if store.check([f"{ar.pacer.prefix}/{r}"]) or store.check([f"{ar.pacer.prefix}/passed/{r}"])]
        if transport == "onesided":
            left = []
        q.put((rank, elapsed, ar.pacer.waits, None if not left else f"pacing keys left for rounds {left}"))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, -1.0, -1, repr(e)))


def _run(th_allreduce, rounds=5, nap=0.3, world=4, transport="reactive"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, th_allreduce, rounds, nap, q, transport))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, r
    return res


@pytest.mark.parametrize("transport", ["reactive", "onesided"])
def test_pacing_advances_without_the_slow_rank(transport):
    rounds, nap = 5, 0.3
    res = _run(0.75, rounds, nap, transport=transport)
    for rank, elapsed, waits, _ in res[:3]:
        assert elapsed < nap * rounds / 2, (rank, elapsed)


@pytest.mark.parametrize("transport", ["reactive", "onesided"])
def test_full_pacing_waits_for_every_rank(transport):
    rounds, nap = 4, 0.3
    res = _run(1.0, rounds, nap, transport=transport)
    for rank, elapsed, waits, _ in res[:3]:
        # round r+1 starts only after the sleeper completed round r (the
        # ranks' clocks start a little apart: 20% slack)
        assert elapsed > 0.8 * nap * (rounds - 1), (rank, elapsed)
        assert waits >= rounds - 2
