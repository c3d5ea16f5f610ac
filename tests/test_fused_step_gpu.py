"""gfx950 kernels of the config-5 training step: the bf16 weight shadow
stored by the fused average + SGD pass, and the bf16 column sum (bias
gradient).  Each compares against a plain torch fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,ncol,off", [(256, 8192, 0), (256, 1000, 0), (37, 1003, 0), (1, 16, 0),
                                        (1000, 24, 8), (64, 520, 3), (5, 4096, 0)])
def test_colsum_matches_torch(M, ncol, off):
    from akka_allreduce_amd.ops import colsum

    g = torch.Generator(device="cuda").manual_seed(M * 7 + ncol)
    base = torch.randn(M * ncol + off, device="cuda", generator=g).to(torch.bfloat16)
    x = base[off:].view(M, ncol)  # off != 0: rows not 16-B aligned (scalar path)
    want = x.float().sum(0)
    for _ in range(3):  # the tickets re-arm: repeated calls on one workspace agree
        got = colsum(x)
        torch.cuda.synchronize()
        torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-4 * max(1.0, M ** 0.5))
    # deterministic: the same input gives bitwise the same sums
    assert torch.equal(colsum(x), colsum(x))


def test_count_mean_shadow_is_bf16_of_updated_params():
    from akka_allreduce_amd.data import AllReduceOutput, Geometry

    S, N, C = 1_000_003, 4, 4099
    g = Geometry(S, N, C)
    d = torch.randn(S, device="cuda")
    pc = torch.randint(0, N + 1, (N, g.kmax), device="cuda", dtype=torch.int32)
    y0 = torch.randn(S, device="cuda")
    want = AllReduceOutput(d, counts_per_chunk=pc, geometry=g).axpy_mean_(y0.clone(), -0.05)
    y = y0.clone()
    shadow = torch.full((S,), 7.0, device="cuda", dtype=torch.bfloat16)
    AllReduceOutput(d, counts_per_chunk=pc, geometry=g).axpy_mean_(y, -0.05, shadow=shadow)
    torch.cuda.synchronize()
    assert torch.equal(y, want)  # the fp32 update is unchanged by the extra store
    assert torch.equal(shadow, y.to(torch.bfloat16))  # RNE, as torch's cast


def test_mlp_bf16_shadow_weights_match_casts():
    """bf16 steps reading the fused update's weight shadow follow bitwise
    the same trajectory as steps that cast the fp32 weights every step; a
    parameter changed in place by torch between steps refreshes the shadow."""
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    x, y = synthetic_batch(64, 256, 10, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    runs = []
    for shadow in (False, True):
        torch.manual_seed(0)
        model = MLP(256, 512, 10).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=4096, device=dev)
        losses = []
        for k in range(6):
            if k == 3:
                with torch.no_grad():
                    model.fc1.weight.mul_(0.5)  # bumps the version: the shadow must be re-copied
            losses.append(dp_sgd_step(model, x, y, 0.1, ar, bucket, compute_dtype=torch.bfloat16,
                                      shadow_weights=shadow))
        assert bucket._shadow_on == shadow
        torch.cuda.synchronize()
        runs.append((losses, [p.detach().clone() for p in model.parameters()], bucket))
    assert runs[0][0] == runs[1][0]
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)
    b = runs[1][2]
    assert torch.equal(b.sflat, b.pflat.to(torch.bfloat16))


@pytest.mark.parametrize("B,C", [(256, 1000), (7, 3), (33, 4099), (1, 1)])
def test_fused_cross_entropy_matches_torch(B, C):
    """Loss and bf16 logit gradient against torch's fp32 cross entropy of the
    same bf16 logits, with a few ignored labels and a non-unit upstream grad."""
    import torch.nn.functional as F

    from akka_allreduce_amd.ops import cross_entropy

    g = torch.Generator(device="cuda").manual_seed(B * 31 + C)
    logits = (4 * torch.randn(B, C, device="cuda", generator=g)).to(torch.bfloat16)
    y = torch.randint(0, C, (B,), device="cuda", generator=g)
    if B > 4:
        y[1] = -100  # ignored rows: excluded from the mean
        y[3] = -100
    for _ in range(2):  # the ticket re-arms
        a = logits.clone().requires_grad_(True)
        loss = cross_entropy(a, y)
        (3.0 * loss).backward()
        r = logits.float().clone().requires_grad_(True)
        want = F.cross_entropy(r, y, ignore_index=-100)
        (3.0 * want).backward()
        torch.testing.assert_close(loss, want, rtol=1e-5, atol=1e-5)
        assert a.grad.dtype == torch.bfloat16
        torch.testing.assert_close(a.grad.float(), r.grad, rtol=1e-2, atol=2e-3 * float(r.grad.abs().max()) + 1e-6)


def test_fused_cross_entropy_flags_invalid_labels():
    """torch ignores only -100 and raises on other out-of-range labels: the
    fused kernel makes the loss NaN, counts the bad rows on the device, and
    AKKA_CHECK_LABELS raises."""
    from akka_allreduce_amd.ops import xent

    logits = torch.randn(8, 5, device="cuda").to(torch.bfloat16)
    y = torch.tensor([0, 1, -100, 4, 7, 2, -3, 1], device="cuda")
    loss = xent.cross_entropy(logits, y)
    assert torch.isnan(loss).item()
    assert xent.last_bad_labels() == 2
    y_ok = torch.tensor([0, 1, -100, 4, 3, 2, 0, 1], device="cuda")
    assert torch.isfinite(xent.cross_entropy(logits, y_ok)).item() and xent.last_bad_labels() == 0
    old = xent._CHECK_LABELS
    xent._CHECK_LABELS = True
    try:
        with pytest.raises(ValueError, match="outside"):
            xent.cross_entropy(logits, y)
    finally:
        xent._CHECK_LABELS = old


def test_mlp_bf16_fused_loss_tracks_torch_loss():
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    x, y = synthetic_batch(64, 256, 10, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    runs = []
    for fused in (False, True):
        torch.manual_seed(0)
        model = MLP(256, 512, 10).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=4096, device=dev)
        runs.append([dp_sgd_step(model, x, y, 0.1, ar, bucket, compute_dtype=torch.bfloat16, fused_loss=fused)
                     for _ in range(20)])
    a, b = runs
    assert abs(a[0] - b[0]) < 1e-4 * abs(a[0])
    assert b[-1] < 0.5 * b[0]
    assert abs(a[-1] - b[-1]) < 0.05 * abs(a[-1]) + 1e-3


@pytest.mark.parametrize("cdt", [None, torch.bfloat16])
def test_graphed_step_matches_eager(cdt):
    """forward + backward replayed from a HIP graph: same losses and
    parameters as the eager step over several steps with new batches."""
    from akka_allreduce_amd.models.mlp import MLP, GraphedDPStep, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(5)
    batches = [synthetic_batch(64, 256, 10, device=dev, generator=gen) for _ in range(6)]
    runs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        model = MLP(256, 512, 10).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=4096, device=dev)
        if graphed:
            # the warmup/capture runs forward+backward only: parameters unchanged
            step = GraphedDPStep(model, bucket, *batches[0], compute_dtype=cdt)
            losses = [float(step(x, y, 0.1, ar)) for x, y in batches]
        else:
            losses = [dp_sgd_step(model, x, y, 0.1, ar, bucket, compute_dtype=cdt) for x, y in batches]
        torch.cuda.synchronize()
        runs.append((losses, [p.detach().clone() for p in model.parameters()]))
    for a, b in zip(runs[0][0], runs[1][0]):
        assert abs(a - b) <= 1e-5 * abs(a) + 1e-6, (runs[0][0], runs[1][0])
    for a, b in zip(runs[0][1], runs[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("M,ncol,off", [(256, 8192, 0), (37, 1003, 0), (64, 520, 3)])
def test_colsum_fused_relu_backward_matches_torch(M, ncol, off):
    """colsum(relu_of=h): the ReLU backward (dY where h > 0, else 0) written
    bitwise like torch's threshold_backward, and its column sums."""
    from akka_allreduce_amd.ops import colsum

    g = torch.Generator(device="cuda").manual_seed(M + ncol)
    base = torch.randn(M * ncol + off, device="cuda", generator=g).to(torch.bfloat16)
    dy = base[off:].view(M, ncol)
    h = torch.relu(torch.randn(M, ncol, device="cuda", generator=g)).to(torch.bfloat16)
    masked = torch.empty(M, ncol, device="cuda", dtype=torch.bfloat16)
    got = colsum(dy, relu_of=h, masked_out=masked)
    want_masked = torch.ops.aten.threshold_backward(dy, h, 0)
    torch.cuda.synchronize()
    assert torch.equal(masked, want_masked)
    torch.testing.assert_close(got, want_masked.float().sum(0), rtol=1e-5, atol=1e-4 * max(1.0, M ** 0.5))
