"""Same-box A/B of BASELINE config 5's EAGER step between two trees of this
framework (``--root``: the tree whose package is imported, e.g. the round-1
tree checked out under ab/r01 with its own in-tree extension).  The step is
bench.py's: MLP 4096-8192-1000, batch 256, flat gradient bucket, N=1
ThresholdAllreduce, ``dp_sgd_step(..., sync_loss=False)``, fp32 and bf16
autocast.  Prints one JSON line: steps/s (device-synchronised around K steps,
after W warm-up steps) and host µs per step (the time to ISSUE the K steps,
measured separately with a synchronise only at the end -- the step is
host-bound when that is close to the step time).

    python bench/cfg5_ab.py --root ab/r01 --steps 50
"""
import argparse
import json
import os
import sys
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtypes", default="fp32,bf16")
    a = ap.parse_args()
    root = os.path.abspath(a.root)
    sys.path.insert(0, root)
    import torch

    import akka_allreduce_amd
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    assert os.path.dirname(os.path.dirname(os.path.abspath(akka_allreduce_amd.__file__))) == root
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    d_in, hidden, classes, batch = 4096, 8192, 1000, 256
    model = MLP(d_in, hidden, classes).to(dev)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=(4 << 20) // 4, device=dev, rank=0, world_size=1)
    xb, yb = synthetic_batch(batch, d_in, classes, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    res = {"root": os.path.relpath(root, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
           "steps": a.steps}
    for name in a.dtypes.split(","):
        cdt = torch.bfloat16 if name == "bf16" else None

        def step():
            return dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False, compute_dtype=cdt)

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        host = time.perf_counter() - t0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name] = {"steps_per_s": round(a.steps / dt, 1), "ms_per_step": round(dt / a.steps * 1e3, 4),
                     "host_us_per_step": round(host / a.steps * 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
