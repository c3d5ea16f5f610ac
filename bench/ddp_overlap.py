"""torch DDP with the threshold comm hook on the one-sided lane: bucket
rounds synchronous on the caller's stream vs async on the lane's side stream
(overlapping the rest of backward).  torch.distributed.run, ranks on the
box's GPU(s); prints one JSON line per mode from rank 0."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--cu-keep", type=int, default=6)
    ap.add_argument("--transport", default="onesided", choices=["onesided", "stream"])
    ap.add_argument("--data-plane", default="ipc", help="stream transport: rccl | ipc")
    ap.add_argument("--modes", default="sync,async", help="comma list (one process per mode avoids the second "
                                                          "mode inheriting the first one's engines and windows)")
    ap.add_argument("--bucket-view", type=int, default=1, help="DDP gradient_as_bucket_view (1: grads are views "
                                                                  "of the buckets, the hook's in-place mean needs no copy)")
    ap.add_argument("--window-output", type=int, default=0, help="onesided: exact rounds return the lane's window row "
                                                                      "(no gather copy)")
    ap.add_argument("--lane", default="", help="stream transport: the hook's lane for every bucket engine "
                                                  "(ThresholdAllreduce.LANES), e.g. ipc_fused_lite")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0 if os.environ.get("AKKA_SHARE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.models.mlp import MLP, synthetic_batch
    from akka_allreduce_amd.parallel.ddp import ThresholdHookState, threshold_allreduce_hook

    for mode in a.modes.split(","):
        torch.manual_seed(0)
        model = torch.nn.parallel.DistributedDataParallel(MLP(4096, 8192, 1000).to(dev), device_ids=[dev.index],
                                                          bucket_cap_mb=a.bucket_mb,
                                                          gradient_as_bucket_view=bool(a.bucket_view))
        state = ThresholdHookState(transport=a.transport, max_chunk_size=1 << 20, async_op=(mode == "async"),
                                   bucket_cap_mb=a.bucket_mb, onesided_options={"cu_keep": a.cu_keep,
                                                                    "window_output": bool(a.window_output)},
                                   data_plane=a.data_plane if a.transport == "stream" else "rccl")
        if a.lane:
            state.lane = a.lane  # applied to every bucket's engine (ThresholdHookState.engine)
        model.register_comm_hook(state, threshold_allreduce_hook)
        opt = torch.optim.SGD(model.parameters(), lr=0.05)
        g = torch.Generator(device=dev).manual_seed(100 + rank)
        x, y = synthetic_batch(256, 4096, 1000, device=dev, generator=g)

        def step():
            opt.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(model(x), y).backward()
            opt.step()

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t = [None] * world
        dist.all_gather_object(t, dt)
        errs = [ar._os.error() if ar.transport == "onesided" else ar.ipc_error() for ar in state.engines.values()]
        if rank == 0:
            print(json.dumps({"mode": mode, "transport": a.transport, "lane": a.lane or None, "world": world,
                              "bucket_view": bool(a.bucket_view),
                              "ms_per_step": round(max(t) / a.steps * 1e3, 3),
                              "buckets": len(state.engines), "async_rounds": state.async_rounds,
                              "rounds": state.rounds, "lane_errors": errs}), flush=True)
        del model, state, opt
        torch.cuda.synchronize()
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
