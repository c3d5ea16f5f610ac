"""Rank program for tests/test_dp_ipc_gpu.py (torch.distributed.run): data-
parallel SGD of the 2-layer MLP (BASELINE config 5's model, smaller) with
every rank on the same GPU and the gradient allreduce on the ipc-only data
plane -- N real processes, real GPU gradients, real cross-process rounds.
Saves the final flat parameters to <out>/rank<i>.pt."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--bf16", action="store_true")
    a = ap.parse_args()
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    torch.manual_seed(0)  # identical init on every rank
    model = MLP(256, 512, 10).to(dev)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=1 << 14, device=dev, data_plane="ipc")
    losses = []
    rec = []  # every round's input and output, for the test's diagnosis on a mismatch

    def recording_ar(t):
        xin = t.detach().clone()
        o = ar(t)
        rec.append((xin, o.data.detach().clone()))  # (not o.count: it would bypass the fused update)
        return o

    for s in range(a.steps):
        g = torch.Generator(device=dev).manual_seed(100 * s + rank)
        x, y = synthetic_batch(64, 256, 10, device=dev, generator=g)
        loss = dp_sgd_step(model, x, y, 0.1, recording_ar, bucket, compute_dtype=torch.bfloat16 if a.bf16 else None)
        losses.append(float(loss))
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])
    torch.save({"flat": flat, "losses": losses, "ipc_error": ar.ipc_error(),
                "ipc_rounds": ar.state()["link"]["ipc_rounds"],
                "rounds_in": [r[0].cpu() for r in rec], "rounds_out": [r[1].cpu() for r in rec]}, os.path.join(a.out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
