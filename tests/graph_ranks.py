"""Rank program for tests/test_graph_step_gpu.py: the 2-layer MLP's DP-SGD
step with the WHOLE step (forward, backward, the one-sided allreduce and the
fused average + SGD update) captured in one HIP graph, against the eager step
on the same batches (every rank on the box's one GPU).  Writes rank<i>.pt."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--lane", default="onesided", choices=["onesided", "ipc"])
    a = ap.parse_args()
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.models.mlp import MLP, GraphedDPStep, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel.dp import GradientBucket
    from akka_allreduce_amd.parallel.onesided import OneSidedAllreduce

    cdt = torch.bfloat16 if a.dtype == "bf16" else None
    lr = 0.05

    def batches():
        for s in range(a.steps):
            g = torch.Generator(device=dev).manual_seed(1000 * s + rank)
            yield synthetic_batch(64, 256, 10, device=dev, generator=g)

    def fresh():
        torch.manual_seed(0)
        m = MLP(256, 512, 10).to(dev)
        return m, GradientBucket(list(m.parameters()), flatten_params=True)

    m1, b1 = fresh()
    if a.lane == "onesided":
        ar = OneSidedAllreduce(b1.numel, max_chunk_size=1 << 14, device=dev)
        cap = ar
    else:
        # the engine's ipc lane: eager steps through the engine, graphed
        # steps through its capturable view (device round ids)
        from akka_allreduce_amd.parallel import ThresholdAllreduce

        ar = ThresholdAllreduce(b1.numel, max_chunk_size=1 << 14, device=dev, data_plane="ipc")
        ar.use_lane("ipc_fused_lite")
    eager_losses = []
    for x, y in batches():
        eager_losses.append(dp_sgd_step(m1, x, y, lr, ar, b1, sync_loss=False, compute_dtype=cdt))
    eager = b1.pflat.clone()

    m2, b2 = fresh()
    x0, y0 = next(batches())
    if a.lane == "ipc":
        torch.cuda.synchronize()
        cap = ar.capturable()
    gs = GraphedDPStep(m2, b2, x0, y0, compute_dtype=cdt, allreduce=cap, lr=lr)
    sx, sy = gs.static_inputs()
    graph_losses = []
    calls0 = ar.calls if a.lane == "onesided" else 0
    for x, y in batches():
        sx.copy_(x)
        sy.copy_(y)
        graph_losses.append(gs(sx, sy, lr, None).clone())
    torch.cuda.synchronize()
    graphed = b2.pflat.clone()
    if a.lane == "onesided":
        st = ar.stats()
        extra = {"calls": ar.calls - calls0, "error": ar.error(), "forced": st["complete_forced"]}
        # an eager call after the captured ones: the host's call ids stayed in
        # step with the device's call sequence (the capture itself ran no
        # call), so this call's record is found and names its round
        w = dist.get_world_size()
        o = ar(torch.full((b1.numel,), float(rank + 1), device=dev))
        extra.update({"eager_after_round": o.iteration, "eager_after_call": o.call, "calls_total": ar.calls,
                      "eager_after_exact": bool((o.data == w * (w + 1) / 2).all().item())})
    else:
        r_after = ar.worker._core.ipc_current_round()
        cap.close()
        extra = {"calls": 20, "error": ar.ipc_error(), "forced": 0, "device_round": r_after}
    torch.save({"eager": eager.cpu(), "graphed": graphed.cpu(), "eager_losses": torch.stack(eager_losses).cpu(),
                "graph_losses": torch.stack(graph_losses).cpu(), "replays": gs.replays, **extra},
               os.path.join(a.out_dir, f"rank{rank}.pt"))
    ar.retire()
    torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
