"""Where a one-sided round's time goes: per-role spans from the kernel's
per-workgroup wall-clock stamps (AKKA_OS_TIMELINE=1; [entry, round known,
role done] per workgroup).  torch.distributed.run, exact rounds; prints one
JSON line per (rank, size): microseconds from the earliest workgroup entry."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["AKKA_OS_TIMELINE"] = "1"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def spans(tl, info, khz):
    g = info["role_wgs"]
    kme = info["kme"]
    bounds = [("begin", 1), ("push", g["push"]), ("decide", kme), ("reduce", g["reduce"]), ("complete", 1),
              ("copy", g["copy"])]
    t = [tl[i:i + 3] for i in range(0, len(tl), 3)]
    n = sum(c for _, c in bounds)
    t = t[:n]
    t0 = min(w[0] for w in t)
    us = lambda v: round((v - t0) * 1e3 / khz, 1)  # noqa: E731
    out, i = {}, 0
    for name, c in bounds:
        ws = t[i:i + c]
        i += c
        if not ws:
            continue
        done = sorted(w[2] for w in ws)
        out[name] = {"first_entry": us(min(w[0] for w in ws)), "round_known": us(max(w[1] for w in ws)),
                     "median_done": us(statistics.median(done)), "last_done": us(done[-1])}
    out["kernel"] = us(max(w[2] for w in t))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="64,256")
    ap.add_argument("--chunk-mb", type=float, default=4.0)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--window-output", action="store_true", help="calls without out: the lane's window row")
    ap.add_argument("--part-bytes", type=int, default=0, help="0: the lane default part size")
    a = ap.parse_args()
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.parallel.onesided import OneSidedAllreduce

    rows = []
    for mb in [float(s) for s in a.sizes_mb.split(",")]:
        S = int(mb * (1 << 20)) // 4
        C = min(S, int(a.chunk_mb * (1 << 20)) // 4)
        ar = OneSidedAllreduce(S, max_chunk_size=C, device=dev, window_output=a.window_output,
                               part_bytes=a.part_bytes)
        info = ar.info()
        info["kme"] = ar.geometry.num_chunks(rank)
        x = torch.randn(S, device=dev)
        out = None if a.window_output else torch.empty_like(x)
        for _ in range(3):
            ar(x, out=out)
        torch.cuda.synchronize()
        per = []
        for _ in range(a.calls):
            dist.barrier()
            ar(x, out=out)
            torch.cuda.synchronize()
            per.append(spans(ar.lane.timeline(), info, info["clock_khz"]))
        best = min(per, key=lambda s: s["kernel"])
        rows.append({"rank": rank, "size_mb": mb, "window_output": ar.window_output, "role_wgs": info["role_wgs"],
                     "kme": info["kme"],
                     "kernel_us_per_call": [s["kernel"] for s in per], "fastest_call": best})
        dist.barrier()
        del ar
    with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(rows, f)
    for r in rows:
        print(json.dumps(r), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
