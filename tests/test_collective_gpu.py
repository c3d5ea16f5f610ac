"""Scheduled (stream) transport on one MI355X: N=1 rounds end to end, plus the
2-layer MLP DP-SGD loop through the worker."""
import pytest
import torch

from akka_allreduce_amd.parallel import ThresholdAllreduce

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("S,C", [(1, 1), (1000, 7), (1 << 20, 1 << 16), ((1 << 22) + 5, 1 << 20)])
def test_single_rank_rounds(dtype, S, C):
    dev = torch.device("cuda", 0)
    ar = ThresholdAllreduce(S, max_chunk_size=C, dtype=dtype, device=dev, rank=0, world_size=1)
    for r in range(5):
        x = (torch.randn(S, device=dev) * (r + 1)).to(dtype)
        out = ar(x)
        assert out.iteration == r
        assert torch.equal(out.data, x)
        assert bool((out.count == 1).all())
    st = ar.state()
    assert st["round"] == 5 and st["stats"]["rounds_completed"] == 5


def test_output_stream_ordering_under_reuse():
    """The output must be valid in the caller's stream even when inputs are
    overwritten right after the call (stream-ordered hand-off)."""
    dev = torch.device("cuda", 0)
    S = 1 << 22
    ar = ThresholdAllreduce(S, max_chunk_size=1 << 18, device=dev, rank=0, world_size=1, max_lag=1)
    x = torch.zeros(S, device=dev)
    outs = []
    for r in range(6):
        x.fill_(float(r))
        outs.append(ar(x))
    for r, o in enumerate(outs):
        assert bool((o.data == float(r)).all()), r


def test_async_rounds_pipeline():
    """async_op rounds: no per-round stream hop; results valid after wait()."""
    dev = torch.device("cuda", 0)
    S = (1 << 22) + 3
    ar = ThresholdAllreduce(S, max_chunk_size=1 << 20, device=dev, rank=0, world_size=1, max_lag=2)
    xs = [torch.full((S,), float(r), device=dev) for r in range(8)]
    outs = [ar(x, async_op=True) for x in xs]
    for r, o in enumerate(outs):
        o.wait()
        assert bool((o.data == float(r)).all()), r
        assert bool((o.count == 1).all())


def test_mlp_dp_sgd_through_allreduce():
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = MLP(64, 128, 10).to(dev)
    bucket = GradientBucket(list(model.parameters()))
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=4096, device=dev, rank=0, world_size=1)
    x, y = synthetic_batch(256, 64, 10, device=dev)
    losses = [dp_sgd_step(model, x, y, 0.5, ar, bucket) for _ in range(60)]
    assert losses[-1] < 0.5 * losses[0], losses


def test_mlp_dp_sgd_bf16_autocast_tracks_fp32():
    """bf16 GEMMs (autocast) with fp32 weights/grads/allreduce: the fused
    count-mean + SGD bucket still trains, and the first step's update matches
    the fp32 step to bf16 tolerance."""
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    runs = {}
    for cdt in (torch.float32, torch.bfloat16):
        torch.manual_seed(0)
        model = MLP(64, 128, 10).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=4096, device=dev, rank=0, world_size=1)
        x, y = synthetic_batch(256, 64, 10, device=dev)
        losses = [dp_sgd_step(model, x, y, 0.5, ar, bucket, compute_dtype=cdt) for _ in range(60)]
        assert all(p.dtype == torch.float32 for p in model.parameters())
        runs[cdt] = losses
    f32, b16 = runs[torch.float32], runs[torch.bfloat16]
    assert abs(b16[0] - f32[0]) < 2e-2 * abs(f32[0]), (b16[0], f32[0])
    assert b16[-1] < 0.5 * b16[0], b16


def test_mlp_bf16_direct_grads_match_autocast_autograd():
    """The bf16 direct-into-bucket backward (_LinearIntoBucket under autocast,
    fp32-out GEMM) gives the same fc1/fc2 weight AND bias gradients as
    autocast + autograd's zero/accumulate path, to bf16 tolerance."""
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    grads = {}
    for direct in (True, False):
        torch.manual_seed(0)
        model = MLP(256, 512, 10).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        x, y = synthetic_batch(128, 256, 10, device=dev)
        bucket.flat.fill_(7.0)  # stale values: the direct path must overwrite every element
        dp_sgd_step(model, x, y, 0.0, None, bucket, compute_dtype=torch.bfloat16, direct_grads=direct)
        assert model.last_step_direct == direct
        grads[direct] = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    assert set(grads[True]) == {"fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"}
    for name in grads[True]:
        a, b = grads[True][name], grads[False][name]
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-3 * float(b.abs().max()) + 1e-6, msg=name)


def test_round_captured_in_hip_graph():
    """An exact-threshold round with fixed buffers captured with
    torch.cuda.graph (relaxed mode) replays the same GPU work: new input
    values written before replay() show up summed in the output."""
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    S = 100_003
    ar = ThresholdAllreduce(S, max_chunk_size=4096, device=torch.device("cuda", 0))
    x = torch.randn(S, device="cuda")
    buf = torch.empty(S, device="cuda")
    ar(x, out=buf)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            for _ in range(3):
                out = ar(x, out=buf)
    for k in range(3):
        x.copy_(torch.full((S,), float(k + 1), device="cuda"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out.data, x) and bool((out.count == 1).all())


def test_fused_average_sgd_matches_unfused():
    """GradientBucket(flatten_params=True): the count-mean + SGD update in one
    pass gives the same training trajectory as average() + sgd_step()."""
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    x, y = synthetic_batch(64, 256, 10, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    params = []
    for fused in (False, True):
        torch.manual_seed(0)
        model = MLP(256, 512, 10).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=fused)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=4096, device=dev)
        for _ in range(5):
            dp_sgd_step(model, x, y, 0.1, ar, bucket, sync_loss=False)
        torch.cuda.synchronize()
        params.append([p.detach().clone() for p in model.parameters()])
    for a, b in zip(*params):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_axpy_mean_matches_torch():
    from akka_allreduce_amd.data import AllReduceOutput, Geometry

    S, N, C = 100_003, 4, 999
    g = Geometry(S, N, C)
    d = torch.randn(S, device="cuda")
    pc = torch.randint(0, N + 1, (N, g.kmax), device="cuda", dtype=torch.int32)
    y = torch.randn(S, device="cuda")
    want = y + (-0.05) * AllReduceOutput(d, counts_per_chunk=pc, geometry=g).mean()
    got = AllReduceOutput(d, counts_per_chunk=pc, geometry=g).axpy_mean_(y.clone(), -0.05)
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("async_op", [False, True])
def test_fast_path_matches_callback_path(async_op):
    """ThresholdAllreduce rounds bind their buffers natively (no Python
    callbacks per round); a worker with a user data source takes the callback
    path.  Both give the same outputs and counts, round after round."""
    from akka_allreduce_amd import AllreduceWorker, InitWorkers

    dev = torch.device("cuda", 0)
    S, C = (1 << 18) + 3, 1 << 14
    xs = [torch.randn(S, device=dev) for _ in range(4)]
    ar = ThresholdAllreduce(S, max_chunk_size=C, device=dev, rank=0, world_size=1)
    assert ar.worker._fast_ok(xs[0])
    fast = [ar(x, async_op=async_op) for x in xs]
    assert not ar.worker._fast_pending

    got = []
    w = AllreduceWorker(lambda req: xs[req.iteration], got.append, device=dev, transport="stream", strict=True)
    w.tell(InitWorkers({0: w}, 1, None, 0, 1.0, 1.0, 2, S, C))
    assert not w._fast_ok(xs[0])  # user data source: callback path
    for r in range(len(xs)):
        w.allreduce(xs[r])
    for r, (a, b) in enumerate(zip(fast, got)):
        a.wait()
        assert a.iteration == b.iteration == r
        assert torch.equal(a.data, xs[r]) and torch.equal(b.data, xs[r])
        assert torch.equal(a.count, b.count) and bool((a.count == 1).all())
