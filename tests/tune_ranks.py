"""Rank program for tests/test_tune_burst.py: ThresholdAllreduce.tune() over
explicit candidates on CPU processes (gloo), one JSON record per rank with
tune()'s result and a few rounds on the chosen lane.  Run under
torch.distributed.run."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--candidates", default="onesided,onesided_fenced")
    ap.add_argument("--size", type=int, default=4099)
    ap.add_argument("--chunk", type=int, default=512)
    ap.add_argument("--dtype", default="float32")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    dtype = torch.bfloat16 if a.dtype == "bfloat16" else torch.float32
    ar = ThresholdAllreduce(a.size, max_chunk_size=a.chunk, dtype=dtype, device="cpu")
    res = ar.tune(candidates=a.candidates.split(","), rounds=2)
    exact = []
    for k in range(3):  # rounds on the chosen lane afterwards
        x = torch.full((a.size,), float((rank + 1) * (k + 1)), dtype=dtype)
        o = ar(x)
        exact.append(bool(torch.all(o.data == (k + 1) * world * (world + 1) // 2).item()))
    with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"rank": rank, "tune": res, "exact_after": exact, "state_lane": ar.state()["link"].get("lane")}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
