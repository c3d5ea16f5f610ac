"""Host cost of one OneSidedAllreduce call vs one engine (ThresholdAllreduce)
call on the ipc lane, as the DDP hook makes them: enqueue only (no sync),
small buffer so the GPU never holds the host back.  torch.distributed.run,
ranks on the box's GPU; rank 0 prints one JSON line per lane."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", default="onesided,engine_ipc_fused_lite,direct_ipc_fused_lite")
    ap.add_argument("--calls", type=int, default=300)
    args = ap.parse_args()
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    S, calls = 1 << 16, args.calls
    x = torch.randn(S, device=dev)
    for name, kw, lane in (("onesided", {"transport": "onesided"}, None),
                           ("engine_ipc_fused_lite", {"data_plane": "ipc"}, "ipc_fused_lite"),
                           ("direct_ipc_fused_lite", {"data_plane": "ipc"}, "ipc_fused_lite_direct")):
        if name not in args.lanes.split(","):
            continue
        ar = ThresholdAllreduce(S, max_chunk_size=1 << 14, device=dev, **kw)
        if lane:
            ar.enable_ipc()
            ar.use_lane(lane)
        for _ in range(20):
            ar(x).mean()
        torch.cuda.synchronize()
        dist.barrier()
        t_call = t_mean = 0.0
        t0 = time.perf_counter()
        for _ in range(calls):
            a = time.perf_counter()
            o = ar(x)
            b = time.perf_counter()
            o.mean()
            t_call += b - a
            t_mean += time.perf_counter() - b
        host = time.perf_counter() - t0
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
        if rank == 0:
            print(json.dumps({"lane": name, "host_us_per_call": round(t_call / calls * 1e6, 1),
                              "host_us_per_mean": round(t_mean / calls * 1e6, 1),
                              "host_loop_us": round(host / calls * 1e6, 1), "total_us": round(total / calls * 1e6, 1)}),
                  flush=True)
        dist.barrier()
        del ar
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
