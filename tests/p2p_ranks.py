"""Rank program for tests/test_ipc_p2p_gpu.py (torch.distributed.run): every
rank on the box's one GPU, the transports' grouped send/recv over mapped
mailboxes (csrc/transport/ipc_p2p.cpp) instead of RCCL -- so the scheduled and
the straggler-tolerant schedules run across real processes.  Rank r
contributes 2**r everywhere, so a chunk's value names the exact set of ranks
summed into it.  Writes <out>/rank<i>.json."""
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
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--transport", default="stream", choices=["stream", "reactive"])
    ap.add_argument("--lane", default="auto")
    ap.add_argument("--unit-bytes", type=int, default=-1)
    ap.add_argument("--th", type=float, default=1.0)
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--chunk", type=int, default=1 << 16)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--max-lag", type=int, default=1)
    ap.add_argument("--straggler-ms", type=float, default=0.0, help="the last rank sleeps this long before each round")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    ar = ThresholdAllreduce(a.size, max_chunk_size=a.chunk, th_reduce=a.th, th_complete=a.th, max_lag=a.max_lag,
                            device=dev, transport=a.transport, data_plane="ipc_p2p")
    if a.transport == "stream":
        ar.set_lane(a.lane)
        ar.set_exact_unit_bytes(a.unit_bytes)
    if a.transport == "reactive":
        ar.worker.reactive_timeout = 120.0
    x = torch.full((a.size,), float(2 ** rank), device=dev)
    res = {"rank": rank, "rounds": []}
    t_fast = []
    for r in range(a.rounds):
        if a.straggler_ms and rank == world - 1:
            time.sleep(a.straggler_ms / 1e3)
        t0 = time.perf_counter()
        o = ar(x)
        data = o.data.float().cpu()
        cnt = o.count.cpu()
        t_fast.append(time.perf_counter() - t0)
        v = data.to(torch.int64)
        pop = torch.zeros_like(v)
        for b in range(world):
            pop += (v >> b) & 1
        res["rounds"].append({
            "all": bool((v == 2 ** world - 1).all()),
            "count_matches_members": bool((pop == cnt).all() & (data == v.float()).all()),
            "min_count": int(cnt.min()), "max_count": int(cnt.max()),
            "min_nonzero_count": int(cnt[cnt > 0].min()) if bool((cnt > 0).any()) else 0,
            "frac_present": float((cnt > 0).float().mean()),
            "has_self": bool(((v >> rank) & 1).all()) if a.th >= 1 else None,
        })
    res["ms_per_round"] = [round(t * 1e3, 3) for t in t_fast]
    st = ar.state()
    res["link"] = {k: v for k, v in st.get("link", {}).items() if isinstance(v, (int, float, str))}
    if a.transport == "reactive":
        ar.drain(60.0)
    torch.cuda.synchronize()
    with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
