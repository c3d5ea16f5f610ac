"""Rank program for tests/test_dp_ipc_gpu.py::test_torch_ddp_hook_multiprocess:
torch DistributedDataParallel (gloo process group, every rank on the box's one
GPU) with the threshold-allreduce comm hook on the ipc-only data plane.
Saves the final flat parameters to <out>/rank<i>.pt."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def build_model(name: str) -> torch.nn.Module:
    """``mlp``: the 2-layer MLP.  ``deep``: 3 linear layers (~1.6 MB); with a
    0.3 MB bucket cap DDP's buckets take 3 distinct sizes over the first steps
    (before and after its bucket rebuild) -> 3 bucket engines per hook."""
    from akka_allreduce_amd.models.mlp import MLP

    if name == "mlp":
        return MLP(256, 512, 10)
    return torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.ReLU(), torch.nn.Linear(512, 512),
                               torch.nn.ReLU(), torch.nn.Linear(512, 10))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--model", choices=["mlp", "deep"], default="mlp")
    ap.add_argument("--bucket-mb", type=float, default=0.25)
    ap.add_argument("--transport", choices=["stream", "onesided"], default="stream")
    ap.add_argument("--cu-keep", type=int, default=0, help="onesided: CUs kept of every 8 (bounded footprint)")
    ap.add_argument("--th", type=float, default=1.0, help="onesided: th_reduce = th_complete")
    a = ap.parse_args()
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.models.mlp import synthetic_batch
    from akka_allreduce_amd.parallel.ddp import ThresholdHookState, threshold_allreduce_hook

    torch.manual_seed(0)
    model = torch.nn.parallel.DistributedDataParallel(build_model(a.model).to(dev), device_ids=[0],
                                                      bucket_cap_mb=a.bucket_mb)
    th = {"th_reduce": a.th, "th_complete": a.th, "max_lag": 1} if a.th < 1.0 else {}
    state = ThresholdHookState(data_plane="ipc", max_chunk_size=1 << 14, tune=a.tune, transport=a.transport,
                               onesided_options={"cu_keep": a.cu_keep} if a.cu_keep else None, **th)
    model.register_comm_hook(state, threshold_allreduce_hook)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    import time

    times = []
    for s in range(a.steps):
        t0 = time.perf_counter()
        g = torch.Generator(device=dev).manual_seed(100 * s + rank)
        x, y = synthetic_batch(64, 256, 10, device=dev, generator=g)
        opt.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(model(x), y).backward()
        opt.step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])
    if a.transport == "onesided":  # one lane (window set) per bucket size
        errs = [ar._os.error() for ar in state.engines.values()]
        windows = list(state.engines)
    else:
        errs = [ar.ipc_error() for ar in state.engines.values()]
        windows = sorted({ar.state()["link"]["ipc"]["windows_id"] for ar in state.engines.values()})
    # tuned once per hook (the first engine), every engine on the chosen lane
    chosen = [state.lane] if a.tune else []
    lane_cus = [int(ar._os.info().get("lane_cus", 0)) for ar in state.engines.values()] \
        if a.transport == "onesided" else []
    # the process's lanes share ONE CU-masked stream (a hardware queue each)
    cu_streams = sorted({int(ar._os.lane.cu_stream()) for ar in state.engines.values()}) \
        if a.transport == "onesided" else []
    torch.save({"flat": flat, "buckets": len(state.engines), "rounds": state.rounds, "ipc_errors": errs,
                "async_rounds": state.async_rounds, "lane_cus": lane_cus, "cu_streams": cu_streams,
                "step_s": times,
                "chosen": chosen, "transports": state.transports(), "window_sets": len(windows)},
               os.path.join(a.out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
