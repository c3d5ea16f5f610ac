"""2-layer MLP DP-SGD step (BASELINE config 5) on CPU: fp32 and bf16-autocast
compute both train; weights, grads and the update stay fp32."""
import torch

from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
from akka_allreduce_amd.parallel import ThresholdAllreduce
from akka_allreduce_amd.parallel.dp import GradientBucket


def _train(cdt, steps=40):
    torch.manual_seed(0)
    model = MLP(32, 64, 8)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=1024, device=torch.device("cpu"), rank=0, world_size=1)
    x, y = synthetic_batch(128, 32, 8, device="cpu")
    losses = [dp_sgd_step(model, x, y, 0.5, ar, bucket, compute_dtype=cdt) for _ in range(steps)]
    assert all(p.dtype == torch.float32 and p.grad.dtype == torch.float32 for p in model.parameters())
    return losses


def test_direct_bucket_grads_match_autograd():
    """The backward that writes dW/db straight into the bucket views gives
    the same gradients and update as autograd's zero + accumulate path."""
    res = {}
    for direct in (False, True):
        torch.manual_seed(0)
        model = MLP(32, 64, 8)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=1024, device=torch.device("cpu"), rank=0, world_size=1)
        x, y = synthetic_batch(128, 32, 8, device="cpu")
        bucket.flat.fill_(123.0)  # stale garbage: the direct path must overwrite it
        for _ in range(3):
            dp_sgd_step(model, x, y, 0.1, ar, bucket, direct_grads=direct)
        assert model.last_step_direct == direct and model.direct_grads is False
        res[direct] = (bucket.flat.clone(), torch.cat([p.detach().flatten() for p in model.parameters()]))
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(res[True][1], res[False][1], rtol=1e-5, atol=1e-6)


def test_mlp_fp32_and_bf16_autocast_train():
    f32 = _train(torch.float32)
    b16 = _train(torch.bfloat16)
    assert f32[-1] < 0.5 * f32[0], f32
    assert b16[-1] < 0.5 * b16[0], b16
    assert abs(b16[0] - f32[0]) < 2e-2 * abs(f32[0]), (b16[0], f32[0])


def _fresh(seed=0):
    torch.manual_seed(seed)
    model = MLP(32, 64, 8)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=1024, device=torch.device("cpu"), rank=0, world_size=1)
    return model, bucket, ar


def test_backward_after_dp_step_accumulates_like_autograd():
    """Direct-into-bucket grads are scoped to dp_sgd_step: a later loss built
    from two forwards (micro-batch accumulation) gets autograd's gradients."""
    model, bucket, ar = _fresh()
    x, y = synthetic_batch(64, 32, 8, device="cpu")
    dp_sgd_step(model, x, y, 0.1, ar, bucket)
    assert model.last_step_direct
    ref = MLP(32, 64, 8)
    ref.load_state_dict(model.state_dict())
    for m in (model, ref):
        for p in m.parameters():
            p.grad = None
        loss = torch.nn.functional.cross_entropy(m(x[:32]), y[:32]) + torch.nn.functional.cross_entropy(m(x[32:]), y[32:])
        loss.backward()
    for a, b in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)


def test_zero_grad_before_dp_step_still_trains():
    """zero_grad() (set_to_none) detaches .grad from the bucket; dp_sgd_step
    re-attaches the views, so the update uses the real gradients."""
    model, bucket, ar = _fresh()
    x, y = synthetic_batch(128, 32, 8, device="cpu")
    w0 = model.fc1.weight.detach().clone()
    losses = []
    for _ in range(5):
        model.zero_grad()
        assert model.fc1.weight.grad is None
        losses.append(dp_sgd_step(model, x, y, 0.5, ar, bucket))
        assert bucket.bound()
    assert not torch.equal(model.fc1.weight.detach(), w0)
    assert losses[-1] < losses[0], losses


def test_rebind_keeps_foreign_gradient_values():
    model, bucket, _ = _fresh()
    g = torch.randn_like(model.fc2.weight)
    model.fc2.weight.grad = g.clone()
    assert not bucket.bound()
    assert bucket.rebind() and bucket.bound()
    torch.testing.assert_close(model.fc2.weight.grad, g)


def test_colsum_cpu_matches_torch():
    import torch

    from akka_allreduce_amd.ops import colsum

    x = torch.randn(37, 1003).to(torch.bfloat16)
    torch.testing.assert_close(colsum(x), x.float().sum(0), rtol=1e-5, atol=1e-4)
    out = torch.empty(1003)
    assert colsum(x, out=out) is out


def test_bucket_shadow_off_on_cpu():
    """The bf16 weight shadow is a device feature: on the CPU the bucket says
    no and the bf16 step casts as before."""
    import torch

    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel.dp import GradientBucket

    torch.manual_seed(0)
    model = MLP(32, 64, 5)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    assert bucket.params_bound()
    assert not bucket.use_shadow(torch.bfloat16)
    assert bucket.shadow_of(model.fc1.weight) is None
    x, y = synthetic_batch(16, 32, 5, device="cpu")
    dp_sgd_step(model, x, y, 0.1, None, bucket, compute_dtype=torch.bfloat16)
    assert bucket.sflat is None


def test_cross_entropy_cpu_is_torch():
    import torch
    import torch.nn.functional as F

    from akka_allreduce_amd.ops import cross_entropy

    x = torch.randn(5, 7)
    y = torch.tensor([0, 6, 2, 3, 1])
    assert torch.equal(cross_entropy(x, y), F.cross_entropy(x, y))
