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

from ..ops.colsum import colsum
from ..ops.xent import cross_entropy
from ..parallel.dp import AllreduceFn, GradientBucket


def _mm_into(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> None:
    """out <- a @ b, written in place (fp32 out from bf16 operands when the
    GEMM library can; otherwise one cast pass)."""
    if a.dtype == out.dtype:
        torch.mm(a, b, out=out)
        return
    try:
        torch.mm(a, b, out_dtype=out.dtype, out=out)
    except (TypeError, RuntimeError):
        out.copy_(torch.mm(a, b))


class _LinearIntoBucket(torch.autograd.Function):
    """Linear layer whose backward writes dW and db straight into the
    gradient bucket's views (``p.grad``) instead of returning them to
    autograd: no bucket zeroing and no AccumulateGrad read-modify-write pass
    over the 167 MB of gradients per step.  Under autocast the GEMMs run in
    the autocast dtype (bf16 MFMA) and the weight/bias stay fp32; ``ws`` /
    ``bs`` are the bucket's bf16 shadows of w / b (written by the previous
    step's fused update), used instead of casting w / b again."""

    @staticmethod
    def forward(ctx, x, w, b, gw, gb, ws=None, bs=None):
        dt = torch.get_autocast_dtype(x.device.type) if torch.is_autocast_enabled(x.device.type) else None
        with torch.autocast(device_type=x.device.type, enabled=False):
            if dt is not None and ws is not None and bs is not None and ws.dtype == dt and bs.dtype == dt:
                xc, wc, bc = x.to(dt), ws, bs
            elif dt is not None:
                xc, wc, bc = x.to(dt), w.to(dt), b.to(dt)
            else:
                xc, wc, bc = x, w, b
            y = F.linear(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.gw, ctx.gb = gw, gb
        return y

    @staticmethod
    def backward(ctx, go):
        xc, wc = ctx.saved_tensors
        go2 = go.reshape(-1, go.shape[-1]).to(wc.dtype)
        _mm_into(go2.t(), xc.reshape(-1, xc.shape[-1]), ctx.gw)
        if go2.is_cuda and go2.dtype == torch.bfloat16 and ctx.gb.dtype == torch.float32 and ctx.gb.is_contiguous():
            colsum(go2, out=ctx.gb.view(-1))  # gfx950 column sum (ops/colsum.py)
        else:
            torch.sum(go2, 0, dtype=ctx.gb.dtype, out=ctx.gb)
        gx = (go2 @ wc).reshape(*go.shape[:-1], wc.shape[1]) if ctx.needs_input_grad[0] else None
        return gx, None, None, None, None, None, None


class _LinearReluIntoBucket(torch.autograd.Function):
    """``relu(x @ w.T + b)`` under bf16 autocast on the GPU, gradients into the
    bucket like ``_LinearIntoBucket``.  Forward: bias and ReLU in the GEMM's
    epilogue (``torch._addmm_activation``: hipBLASLt's RELU_BIAS epilogue), no
    separate activation kernel.  Backward: the ReLU mask, the masked dY and
    the bias gradient in ONE pass (``colsum(relu_of=...)``, gfx950), then the
    dW GEMM on the masked dY."""

    @staticmethod
    def forward(ctx, x, w, b, gw, gb, ws, bs):
        dt = torch.get_autocast_dtype(x.device.type)
        with torch.autocast(device_type=x.device.type, enabled=False):
            xc = x.to(dt)
            wc = ws if ws is not None else w.to(dt)
            bc = bs if bs is not None else b.to(dt)
            x2 = xc.reshape(-1, xc.shape[-1])
            h = torch._addmm_activation(bc, x2, wc.t(), use_gelu=False)
        ctx.save_for_backward(x2, wc, h)
        ctx.gw, ctx.gb, ctx.xshape = gw, gb, xc.shape
        return h.reshape(*xc.shape[:-1], wc.shape[0])

    @staticmethod
    def backward(ctx, go):
        x2, wc, h = ctx.saved_tensors
        go2 = go.reshape(-1, go.shape[-1]).to(wc.dtype).contiguous()
        g = torch.empty_like(go2)
        colsum(go2, out=ctx.gb.view(-1), relu_of=h, masked_out=g)  # ReLU backward + db fused
        _mm_into(g.t(), x2, ctx.gw)
        gx = (g @ wc).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        return gx, None, None, None, None, None, None


class MLP(nn.Module):
    def __init__(self, d_in: int, d_hidden: int, d_out: int):
        super().__init__()
        self.fc1 = nn.Linear(d_in, d_hidden)
        self.fc2 = nn.Linear(d_hidden, d_out)
        # set by dp_sgd_step for its own forward/backward only (every .grad is
        # a bucket view); reset before it returns
        self.direct_grads = False
        self.last_step_direct = False
        self.shadow_bucket: Optional[GradientBucket] = None  # set with direct_grads when bf16 shadows are current

    def _linear(self, fc: nn.Linear, x: torch.Tensor) -> torch.Tensor:
        if self.direct_grads and torch.is_grad_enabled():
            sb = self.shadow_bucket
            ws = sb.shadow_of(fc.weight) if sb is not None else None
            bs = sb.shadow_of(fc.bias) if sb is not None else None
            return _LinearIntoBucket.apply(x, fc.weight, fc.bias, fc.weight.grad, fc.bias.grad, ws, bs)
        return fc(x)

    def _linear_relu(self, fc: nn.Linear, x: torch.Tensor) -> torch.Tensor:
        if (self.direct_grads and torch.is_grad_enabled() and x.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16 and fc.bias is not None
                and fc.bias.grad is not None and fc.bias.grad.is_contiguous()):
            sb = self.shadow_bucket
            ws = sb.shadow_of(fc.weight) if sb is not None else None
            bs = sb.shadow_of(fc.bias) if sb is not None else None
            return _LinearReluIntoBucket.apply(x, fc.weight, fc.bias, fc.weight.grad, fc.bias.grad, ws, bs)
        return F.relu(self._linear(fc, x))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self._linear(self.fc2, self._linear_relu(self.fc1, x))


def dp_sgd_step(model: nn.Module, x: torch.Tensor, y: torch.Tensor, lr: float,
                allreduce: Optional[AllreduceFn], bucket: Optional[GradientBucket] = None,
                sync_loss: bool = True, compute_dtype: Optional[torch.dtype] = None,
                direct_grads: bool = True, shadow_weights: bool = True, fused_loss: bool = True):
    """forward + backward + gradient allreduce (mean over contributors) + SGD
    update.  With a bucket built with ``flatten_params=True`` the averaging and
    the update are one fused pass.  ``sync_loss=False`` returns the loss as a
    device tensor (no host sync per step).  ``compute_dtype=torch.bfloat16``
    runs the forward/backward GEMMs on bf16 MFMA (autocast) while weights,
    gradients, the allreduce and the update stay fp32; with
    ``shadow_weights`` the fused update also stores the bf16 weight copy the
    next step's GEMMs read (``GradientBucket.use_shadow``), so no step casts
    the fp32 weights again."""
    if bucket is None:
        bucket = getattr(model, "_akka_bucket", None)
        if bucket is None:
            bucket = GradientBucket(list(model.parameters()))
            model._akka_bucket = bucket  # type: ignore[attr-defined]
    loss = _forward_backward(model, x, y, bucket, compute_dtype, direct_grads, shadow_weights, fused_loss)
    bucket.sgd_from(allreduce, lr)
    return float(loss.detach()) if sync_loss else loss.detach()


def _forward_backward(model: nn.Module, x: torch.Tensor, y: torch.Tensor, bucket: GradientBucket,
                      compute_dtype: Optional[torch.dtype], direct_grads: bool, shadow_weights: bool,
                      fused_loss: bool, grad_seed: Optional[torch.Tensor] = None) -> torch.Tensor:
    # zero_grad() (set_to_none) or a reassigned .grad detaches a parameter
    # from the bucket: put the views back, or the allreduce would average a
    # buffer autograd no longer writes
    bucket.rebind()
    direct = isinstance(model, MLP) and direct_grads and bucket.bound() \
        and set(map(id, model.parameters())) == set(map(id, bucket.params))
    try:
        if direct:
            # backward overwrites every bucket view directly: nothing to zero.
            # Only for this step's single forward/backward: any other backward
            # (micro-batch accumulation, a later plain loss.backward()) must
            # accumulate as usual.
            model.direct_grads = True
            # bf16 GEMMs read the bf16 weight copy the last fused update wrote
            lowp = compute_dtype if (shadow_weights and compute_dtype is not None
                                     and compute_dtype != torch.float32) else None
            model.shadow_bucket = bucket if bucket.use_shadow(lowp) else None
        else:
            bucket.use_shadow(None)
            bucket.zero_()
        if compute_dtype is not None and compute_dtype != torch.float32:
            with torch.autocast(device_type=x.device.type, dtype=compute_dtype):
                logits = model(x)
            # bf16 logits: the fused gfx950 loss (ops/xent.py), fp32 inside
            loss = cross_entropy(logits, y) if fused_loss else F.cross_entropy(logits.float(), y)
        else:
            loss = F.cross_entropy(model(x), y)
        loss.backward(grad_seed)  # None: autograd's ones; a graph passes a preallocated seed (no fill kernel)
    finally:
        if isinstance(model, MLP):
            model.direct_grads = False
            model.shadow_bucket = None
            model.last_step_direct = direct
    return loss


class GraphedDPStep:
    """``dp_sgd_step`` with the forward + backward captured once in a HIP
    graph (``torch.cuda.CUDAGraph``): a step is two input copies, one graph
    replay, then the gradient allreduce and the fused average + SGD pass,
    eagerly -- an allreduce with a per-round host protocol (the engine's
    lanes) stays outside the graph.  ``allreduce=`` a capturable one (the
    one-sided lane, ``OneSidedAllreduce``) and ``lr=`` capture the WHOLE
    step: forward, backward, allreduce and update in one replay.  The ~30 launches of
    the forward/backward cost one replay instead of ~10 µs of host time each
    (the step is otherwise host-bound at this size).

    The graph bakes in every buffer: the bucket (gradients written directly
    into it), the parameters, the bf16 shadow and the static batch.  Moving
    any of them (``zero_grad(set_to_none=True)``, reassigning ``p.data``, a
    different batch shape) raises; in-place parameter updates by torch are
    fine (they refresh the shadow before the replay)."""

    def __init__(self, model: "MLP", bucket: GradientBucket, x: torch.Tensor, y: torch.Tensor,
                 compute_dtype: Optional[torch.dtype] = None, shadow_weights: bool = True, warmup: int = 3,
                 allreduce: Optional[AllreduceFn] = None, lr: Optional[float] = None):
        if not (x.is_cuda and isinstance(model, MLP)):
            raise ValueError("GraphedDPStep: an MLP on a GPU")
        if bucket.pflat is None or not bucket.bound() or not bucket.params_bound():
            raise ValueError("GraphedDPStep: needs GradientBucket(flatten_params=True) bound to the model")
        self.model, self.bucket = model, bucket
        self.compute_dtype = compute_dtype
        self.lowp = compute_dtype if (shadow_weights and compute_dtype is not None
                                      and compute_dtype != torch.float32) else None
        # the static batch: write the next batch into these (static_inputs())
        # and the replay reads it in place, no copy.  With bf16 GEMMs the
        # input buffer is bf16 -- the first GEMM reads bf16(x) either way --
        # so a batch is converted once as it is written (what a loader that
        # emits bf16 does), not again inside every replay
        lowx = compute_dtype if (compute_dtype is not None and compute_dtype != torch.float32
                                 and x.is_floating_point() and x.dtype == torch.float32) else None
        self.sx = x.detach().to(lowx) if lowx is not None else x.detach().clone()
        self.sy = y.detach().clone()
        self._seed = torch.ones((), dtype=torch.float32, device=x.device)
        self._ptrs = self._pointers()

        # Whole-step capture: an allreduce whose rounds keep their protocol
        # state on the device (``capturable``: the one-sided lane's call id,
        # round and decisions live in device memory, its launch arguments are
        # the same every call) is captured too, with the fused average + SGD
        # update behind it -- a step is then ONE graph replay.
        self.allreduce = allreduce if (allreduce is not None and getattr(allreduce, "capturable", False)) else None
        if allreduce is not None and self.allreduce is None:
            raise ValueError("GraphedDPStep: this allreduce keeps host-side round state; pass it at call time")
        if self.allreduce is not None and lr is None:
            raise ValueError("GraphedDPStep: a captured update needs its learning rate")
        self.lr = lr
        self._out = torch.empty_like(bucket.flat) if self.allreduce is not None else None
        self.replays = 0

        def fb():
            loss = _forward_backward(model, self.sx, self.sy, bucket, compute_dtype, True, shadow_weights, True,
                                     grad_seed=self._seed)
            if self.allreduce is not None:
                bucket.sgd_from(self.allreduce, float(lr), out_buf=self._out)
            return loss

        # warm up and capture on ONE stream: the kernels' per-stream workspaces
        # (colsum / cross-entropy tickets) are created, and zeroed, by the
        # warmup, so the graph holds no fill for them
        side = torch.cuda.Stream(device=x.device)
        side.wait_stream(torch.cuda.current_stream(x.device))
        # a captured update changes the parameters in the warmup steps: they
        # are put back afterwards (the warmup's rounds still ran on every rank)
        snap = bucket.pflat.clone() if self.allreduce is not None else None
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fb()
        side.synchronize()
        # kept alive: the per-stream workspaces baked into the graph are keyed
        # by this stream's handle, which must not be handed to another stream
        self._side = side
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=side):
            self.loss = fb().detach()
        torch.cuda.current_stream(x.device).wait_stream(side)
        if snap is not None:
            bucket.pflat.copy_(snap)
            if bucket.sflat is not None:
                bucket.sflat.copy_(bucket.pflat)
            bucket._shadow_versions = [p._version for p in bucket.params]
        self._ptrs = self._pointers()  # the shadow exists now

    def static_inputs(self):
        """(x, y) buffers the graph reads: fill them with the next batch and
        pass them to the call to skip the copies."""
        return self.sx, self.sy

    def _pointers(self):
        b = self.bucket
        return (b.flat.data_ptr(), b.pflat.data_ptr(), b.sflat.data_ptr() if b.sflat is not None else 0,
                [p.data_ptr() for p in b.params], [p.grad.data_ptr() if p.grad is not None else 0 for p in b.params])

    def __call__(self, x: torch.Tensor, y: torch.Tensor, lr: float, allreduce: Optional[AllreduceFn],
                 sync_loss: bool = False):
        b = self.bucket
        if self._pointers() != self._ptrs:
            raise RuntimeError("GraphedDPStep: a parameter, gradient or shadow buffer moved since the capture")
        if b.use_shadow(self.lowp) != (self.lowp is not None and b.sflat is not None):
            raise RuntimeError("GraphedDPStep: the bf16 shadow is no longer usable")
        if x.data_ptr() != self.sx.data_ptr():
            self.sx.copy_(x)
        if y.data_ptr() != self.sy.data_ptr():
            self.sy.copy_(y)
        if self.allreduce is not None:
            if allreduce is not None and allreduce is not self.allreduce:
                raise RuntimeError("GraphedDPStep: the step captured another allreduce")
            if lr != self.lr:
                raise RuntimeError(f"GraphedDPStep: the update was captured with lr={self.lr}")
            self.graph.replay()  # forward + backward + allreduce + fused update
            self.replays += 1
            self.allreduce.note_replays(1)
            if b._shadow_on:
                b._shadow_versions = [p._version for p in b.params]
        else:
            self.graph.replay()
            b.sgd_from(allreduce, lr)
        return float(self.loss) if sync_loss else self.loss


def synthetic_batch(batch: int, d_in: int, n_classes: int, *, device, generator: Optional[torch.Generator] = None):
    """Linearly separable synthetic classification data (no dataset download)."""
    x = torch.randn(batch, d_in, device=device, generator=generator)
    w = torch.arange(d_in * n_classes, device=device, dtype=torch.float32).reshape(d_in, n_classes).sin()
    y = (x @ w).argmax(dim=1)
    return x, y
