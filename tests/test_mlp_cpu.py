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


def test_mlp_fp32_and_bf16_autocast_train():
    f32 = _train(torch.float32)
    b16 = _train(torch.bfloat16)
    assert f32[-1] < 0.5 * f32[0], f32
    assert b16[-1] < 0.5 * b16[0], b16
    assert abs(b16[0] - f32[0]) < 2e-2 * abs(f32[0]), (b16[0], f32[0])
