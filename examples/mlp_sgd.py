#!/usr/bin/env python3
"""BASELINE config 5: gradient allreduce inside a 2-layer MLP SGD loop on
synthetic data, one process per MI355X (torchrun), end-to-end steps/s.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 examples/mlp_sgd.py

Each step: forward + backward (grads land in one flat bucket), threshold
allreduce of the bucket over xGMI, average by the per-element contributor
counts, SGD update.  Prints one JSON line from rank 0.  Runs on CPU processes
too (gloo p2p) with --cpu.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--d-in", type=int, default=4096)
    p.add_argument("--hidden", type=int, default=8192)
    p.add_argument("--classes", type=int, default=1000)
    p.add_argument("--batch", type=int, default=256, help="per-rank batch")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--chunk-mb", type=float, default=4.0)
    p.add_argument("--th-reduce", type=float, default=1.0)
    p.add_argument("--th-complete", type=float, default=1.0)
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--compute-dtype", choices=["float32", "bfloat16"], default="float32",
                   help="GEMM dtype (bfloat16: autocast onto bf16 MFMA; weights/grads/allreduce stay fp32)")
    p.add_argument("--transport", choices=["stream", "reactive"], default="stream",
                   help="reactive: straggler-tolerant data path (pair with thresholds < 1)")
    p.add_argument("--graph", action="store_true",
                   help="replay forward + backward from one HIP graph (GraphedDPStep; GPU, stream transport)")
    p.add_argument("--straggler-ms", type=float, default=0.0,
                   help="the last rank sleeps this long before every step (BASELINE config 4)")
    a = p.parse_args()
    if a.transport == "reactive" and not a.cpu:
        os.environ["GPU_MAX_HW_QUEUES"] = "32"  # one stream per peer (read at HIP init)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.cpu:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from akka_allreduce_amd.models.mlp import MLP, GraphedDPStep, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    torch.manual_seed(0)  # identical init on every rank
    model = MLP(a.d_in, a.hidden, a.classes).to(dev)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)  # fused average + SGD
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=int(a.chunk_mb * (1 << 20)) // 4, device=dev,
                            th_reduce=a.th_reduce, th_complete=a.th_complete, transport=a.transport)
    nap = a.straggler_ms / 1e3 if rank == world - 1 and world > 1 else 0.0
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    x, y = synthetic_batch(a.batch, a.d_in, a.classes, device=dev, generator=gen)
    cdt = getattr(torch, a.compute_dtype)
    if a.graph and not a.cpu:
        # the batch lives in the graph's static buffers; a data loader would
        # write each new batch there before the step
        graphed = GraphedDPStep(model, bucket, x, y, compute_dtype=cdt)
        x, y = graphed.static_inputs()

        def step():
            return graphed(x, y, a.lr, ar)
    else:
        def step():
            return dp_sgd_step(model, x, y, a.lr, ar, bucket, sync_loss=False, compute_dtype=cdt)

    def sync():
        ar.drain()  # reactive: finish transfers slower peers still need before a blocking collective
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    losses = []
    for _ in range(a.warmup):
        losses.append(step().clone())
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if nap:
            time.sleep(nap)
        losses.append(step().clone())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    own = time.perf_counter() - t0  # this rank's own time (fast ranks vs the straggler)
    sync()
    dt = time.perf_counter() - t0
    owns = [own]
    if world > 1:
        owns = [None] * world
        dist.all_gather_object(owns, own)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        print(json.dumps({
            "metric": "2-layer MLP DP-SGD steps/s (gradient threshold allreduce)",
            "value": round(a.steps / dt, 3), "unit": "steps/s", "n_gpus": world,
            "samples_per_s": round(a.steps * a.batch * world / dt, 1),
            "grad_bytes": bucket.numel * 4, "loss_first": round(float(losses[0]), 4),
            "loss_last": round(float(losses[-1]), 4),
            "fast_ranks_steps_per_s": round(a.steps / max(owns[:-1] if world > 1 else owns), 3),
            "transport": a.transport, "straggler_ms": a.straggler_ms, "compute_dtype": a.compute_dtype,
            "graph": bool(a.graph and not a.cpu),
            "config": {"d_in": a.d_in, "hidden": a.hidden, "classes": a.classes, "batch_per_rank": a.batch},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
