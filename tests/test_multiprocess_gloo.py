"""Multi-process (world_size 2 and 4) runs of the production step schedule on
CPU: one process per rank, torch.distributed gloo as the p2p transport, the
native engine/StreamLink/data plane unchanged.  Exact sums, counts, bf16,
uneven geometry and several rounds through the ring."""
import os
import socket

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


def _rank_main(rank, world, port, S, C, dtype_name, rounds, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from akka_allreduce_amd.parallel import ThresholdAllreduce

        dtype = getattr(torch, dtype_name)
        ar = ThresholdAllreduce(S, max_chunk_size=C, dtype=dtype, rank=rank, world_size=world,
                                device=torch.device("cpu"), max_lag=1)
        ok = True
        for r in range(rounds):
            x = (torch.arange(S, dtype=torch.float32) % 7 + rank * 3 + r).to(dtype)
            out = ar(x)
            want = sum((torch.arange(S, dtype=torch.float32) % 7 + q_ * 3 + r) for q_ in range(world)).to(dtype)
            ok &= torch.equal(out.data, want) and bool((out.count == world).all()) and out.iteration == r
        st = ar.state()
        ok &= ar.worker.fast_rounds == rounds  # collective calls bind their buffers natively
        q.put((rank, ok, st["round"], st["link"]["groups"]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e), 0))


@pytest.mark.parametrize("world,S,C,dtype", [(2, 1000, 64, "float32"), (4, 4099, 128, "float32"),
                                             (3, 777, 50, "bfloat16"), (4, 5, 1, "float32")])
def test_gloo_multiprocess_schedule(world, S, C, dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, S, C, dtype, 4, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, rnd, groups in res:
        assert ok, (rank, rnd)
        assert rnd == 4
