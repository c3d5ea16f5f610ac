"""BASELINE config 5's step alone, one GPU (no peer: the allreduce is the
local pass): MLP 4096-8192-1000, batch 256, DP-SGD through
ThresholdAllreduce, fp32 or bf16 autocast.  For kernel traces:

    rocprofv3 --kernel-trace --stats -d gpurun_out/cfg5 -- python3 bench/cfg5_step.py --dtype bf16
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-shadow", action="store_true", help="bf16: cast the fp32 weights every step")
    ap.add_argument("--graph", action="store_true", help="forward + backward replayed from a HIP graph")
    ap.add_argument("--no-fused-loss", action="store_true", help="bf16: torch's fp32 cross entropy")
    a = ap.parse_args()
    import torch

    from akka_allreduce_amd.models.mlp import MLP, GraphedDPStep, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = MLP(4096, 8192, 1000).to(dev)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=(4 << 20) // 4, device=dev, rank=0, world_size=1)
    x, y = synthetic_batch(256, 4096, 1000, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    cd = torch.bfloat16 if a.dtype == "bf16" else None
    if a.graph:
        g = GraphedDPStep(model, bucket, x, y, compute_dtype=cd, shadow_weights=not a.no_shadow)
        x, y = g.static_inputs()  # the batch lives in the graph's buffers (a loader would write it there)

        def one():
            g(x, y, 0.05, ar)
    else:
        def one():
            dp_sgd_step(model, x, y, 0.05, ar, bucket, sync_loss=False, compute_dtype=cd,
                        shadow_weights=not a.no_shadow, fused_loss=not a.no_fused_loss)
    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    host = time.perf_counter() - t0  # enqueue time (the GPU runs behind it unless the step is host-bound)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"dtype": a.dtype, "shadow": not a.no_shadow and cd is not None, "graph": a.graph,
                      "fused_loss": not a.no_fused_loss and cd is not None and not a.graph or a.graph and cd is not None,
                      "steps": a.steps, "ms_per_step": round(dt / a.steps * 1e3, 4),
                      "host_ms_per_step": round(host / a.steps * 1e3, 4), "steps_per_s": round(a.steps / dt, 2)}),
          flush=True)


if __name__ == "__main__":
    main()
