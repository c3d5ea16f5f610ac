"""DDP communication hook: the threshold allreduce replaces DDP's bucket
allreduce.  Two CPU processes (gloo); at thresholds 1 training must match
stock DDP (mean over all ranks), bucket by bucket."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(use_hook, rank, world, **hook_kw):
    from torch.nn.parallel import DistributedDataParallel as DDP

    from akka_allreduce_amd.parallel.ddp import ThresholdHookState, threshold_allreduce_hook

    torch.manual_seed(0)
    # ~1.7 MB of parameters; DDP's first bucket is 1 MiB, and after its bucket
    # rebuild (first step) a 0.3 MB cap gives several buckets of different sizes
    model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.ReLU(), torch.nn.Linear(512, 512),
                                torch.nn.ReLU(), torch.nn.Linear(512, 64))
    ddp = DDP(model, bucket_cap_mb=0.3)
    state = None
    if use_hook:
        state = ThresholdHookState(max_chunk_size=4096, **hook_kw)
        ddp.register_comm_hook(state, threshold_allreduce_hook)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(3):
        x = torch.randn(16, 256, generator=g)
        y = torch.randn(16, 64, generator=g)
        opt.zero_grad()
        torch.nn.functional.mse_loss(ddp(x), y).backward()
        opt.step()
    return [p.detach().clone() for p in model.parameters()], state


def _main(rank, world, port, q, hook_kw):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ref, _ = _train(False, rank, world)
        got, st = _train(True, rank, world, **hook_kw)
        ok = all(torch.allclose(a, b, rtol=1e-5, atol=1e-6) for a, b in zip(ref, got))
        q.put((rank, ok, st.rounds, len(st.engines), st.transports()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e), 0, 0))


def _run(hook_kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_main, args=(r, 2, port, q, hook_kw)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    return res


def test_ddp_hook_matches_stock_ddp():
    for rank, ok, rounds, engines, transports in _run({}):
        assert ok, (rank, rounds)
        assert rounds >= 3 and engines >= 3  # one round per bucket per step, >= 3 bucket sizes
        assert transports == 1  # every bucket size's engine rides on ONE transport (communicator)


def test_ddp_hook_onesided_matches_stock_ddp():
    """The hook on the one-sided lane (thresholds 1: every contributor, so
    the same mean as DDP's allreduce); on the CPU the windows are shared
    memory running the GPU kernels' protocol."""
    for rank, ok, rounds, engines, _ in _run({"transport": "onesided"}):
        assert ok, (rank, rounds)
        assert rounds >= 3 and engines >= 3


def test_ddp_hook_reactive_keeps_one_transport_per_engine():
    """Reactive engines issue their phase-2 groups from per-peer streams in a
    timing-dependent order, so the hook never lets two of them share a
    transport: each bucket size gets its own, and training still
    matches stock DDP at thresholds 1 over several bucket sizes."""
    for rank, ok, rounds, engines, transports in _run({"transport": "reactive"}):
        assert ok, (rank, rounds)
        assert rounds >= 3 and engines >= 3
        assert transports == engines


def test_share_transport_refuses_reactive():
    import pytest

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    class _Fake:
        transport = "reactive"

    with pytest.raises(ValueError, match="only the scheduled"):
        ThresholdAllreduce(16, transport="reactive", rank=0, world_size=2, device=torch.device("cpu"),
                           share_transport_with=_Fake())


def _straggler_main(rank, world, port, q, delay_ms, steps):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["AKKA_FAULT_RANK"] = "1"
        os.environ["AKKA_FAULT_DELAY_MS"] = str(delay_ms)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import time

        from torch.nn.parallel import DistributedDataParallel as DDP

        from akka_allreduce_amd.parallel.ddp import ThresholdHookState, threshold_allreduce_hook

        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 8))
        ddp = DDP(model, bucket_cap_mb=0.02, gradient_as_bucket_view=True)
        # thresholds 1/2 of 2 ranks: a round completes on this rank's own data
        state = ThresholdHookState(max_chunk_size=1024, transport="onesided", th_reduce=0.5, th_complete=0.5,
                                   max_lag=1)
        ddp.register_comm_hook(state, threshold_allreduce_hook)
        opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
        g = torch.Generator().manual_seed(100 + rank)
        times = []
        for _ in range(steps):
            x = torch.randn(8, 64, generator=g)
            y = torch.randn(8, 8, generator=g)
            t0 = time.perf_counter()
            opt.zero_grad()
            torch.nn.functional.mse_loss(ddp(x), y).backward()
            opt.step()
            times.append(time.perf_counter() - t0)
        finite = all(bool(torch.isfinite(p).all()) for p in model.parameters())
        errs = [ar._os.error() for ar in state.engines.values()]
        q.put((rank, times, state.rounds, finite, errs))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), 0, False, []))


def test_ddp_hook_onesided_straggler_does_not_hold_the_fast_rank():
    """The straggler case the reference exists for, through torch DDP: rank 1
    sleeps 40 ms before each of its bucket rounds; at thresholds 1/2 the
    one-sided rounds of rank 0 complete on what arrived, so its DDP steps
    (after the first two: engine creation and DDP's bucket rebuild are
    collective) take a small fraction of one straggler delay."""
    delay_ms, steps = 40, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_straggler_main, args=(r, 2, port, q, delay_ms, steps)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    (r0, t0, rounds0, fin0, err0), (r1, t1, rounds1, fin1, err1) = res
    assert isinstance(t0, list) and isinstance(t1, list), res
    assert fin0 and fin1 and rounds0 >= steps and rounds1 >= steps
    fast = sorted(t0[2:])[len(t0[2:]) // 2]  # median of the steady steps
    slow = sorted(t1[2:])[len(t1[2:]) // 2]
    assert slow >= delay_ms / 1e3, (t0, t1)  # the straggler pays its delay per round
    assert fast < 0.25 * delay_ms / 1e3, (fast, t0, t1)  # the fast rank never waits for it
