"""2-layer MLP trained with data-parallel SGD through the threshold allreduce
(BASELINE config 5: "gradient allreduce inside a 2-layer MLP SGD loop on
synthetic data").

The reference ships no model (the library is the primitive a DP
trainer calls); this is the minimal consumer that exercises the data-source /
data-sink contract end to end with real gradients.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel.dp import AllreduceFn, GradientBucket


class MLP(nn.Module):
    def __init__(self, d_in: int, d_hidden: int, d_out: int):
        super().__init__()
        self.fc1 = nn.Linear(d_in, d_hidden)
        self.fc2 = nn.Linear(d_hidden, d_out)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc2(F.relu(self.fc1(x)))


def dp_sgd_step(model: nn.Module, x: torch.Tensor, y: torch.Tensor, lr: float,
                allreduce: Optional[AllreduceFn], bucket: Optional[GradientBucket] = None,
                sync_loss: bool = True, compute_dtype: Optional[torch.dtype] = None):
    """forward + backward + gradient allreduce (mean over contributors) + SGD
    update.  With a bucket built with ``flatten_params=True`` the averaging and
    the update are one fused pass.  ``sync_loss=False`` returns the loss as a
    device tensor (no host sync per step).  ``compute_dtype=torch.bfloat16``
    runs the forward/backward GEMMs on bf16 MFMA (autocast) while weights,
    gradients, the allreduce and the update stay fp32."""
    if bucket is None:
        bucket = getattr(model, "_akka_bucket", None)
        if bucket is None:
            bucket = GradientBucket(list(model.parameters()))
            model._akka_bucket = bucket  # type: ignore[attr-defined]
    bucket.zero_()
    if compute_dtype is not None and compute_dtype != torch.float32:
        with torch.autocast(device_type=x.device.type, dtype=compute_dtype):
            loss = F.cross_entropy(model(x), y)
    else:
        loss = F.cross_entropy(model(x), y)
    loss.backward()
    bucket.sgd_from(allreduce, lr)
    return float(loss.detach()) if sync_loss else loss.detach()


def synthetic_batch(batch: int, d_in: int, n_classes: int, *, device, generator: Optional[torch.Generator] = None):
    """Linearly separable synthetic classification data (no dataset download)."""
    x = torch.randn(batch, d_in, device=device, generator=generator)
    w = torch.arange(d_in * n_classes, device=device, dtype=torch.float32).reshape(d_in, n_classes).sin()
    y = (x @ w).argmax(dim=1)
    return x, y
