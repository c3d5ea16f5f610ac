"""Rank program: whole-round times of the one-sided threshold lane next to the
exact ipc lane, on the same processes (run under torch.distributed.run; on a
1-GPU box every rank drives cuda:0).  Writes rank<i>.json into --out-dir.

Per size (MiB, fp32, 4 MiB chunks unless --chunk-mb):
  * onesided  thresholds 1 (exact; checked once against the fp32 sum), W
              warm-up + K timed rounds, ms per round of this rank;
  * ipc       the exact ipc lane (``--ipc-lane``, default ipc_fused_lite),
              same buffer, same W / K;
  * --straggler: BASELINE config 4 (bench.run_cfg4) on the one-sided lane at
              --cfg4-mb: fast ranks' median ms per round with and without
              rank N-1 sleeping --delay-ms per call.

    python -m torch.distributed.run --nproc-per-node 4 ... bench/onesided_round.py --sizes-mb 64,256 --out-dir d
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _time(fn, warmup: int, steps: int) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    dist.barrier()
    return dt


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="64,256")
    ap.add_argument("--chunk-mb", type=float, default=4.0)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--lanes", default="onesided,ipc")
    ap.add_argument("--ipc-lane", default="ipc_fused_lite")
    ap.add_argument("--threads", type=int, default=0, help="onesided workgroup size (0: the lane's default)")
    ap.add_argument("--straggler", action="store_true")
    ap.add_argument("--cfg4-mb", type=float, default=64.0)
    ap.add_argument("--delay-ms", type=float, default=50.0)
    ap.add_argument("--cfg4-rounds", type=int, default=32)
    ap.add_argument("--out-dir", required=True)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.onesided import OneSidedAllreduce

    res: dict = {"rank": rank, "world": world, "cases": []}
    C = int(a.chunk_mb * (1 << 20)) // 4
    for mb in [float(s) for s in a.sizes_mb.split(",") if s]:
        S = int(mb * (1 << 20)) // 4
        x = torch.randn(S, device=dev, generator=torch.Generator(device=dev).manual_seed(11 + rank))
        out = torch.empty_like(x)
        for lane in a.lanes.split(","):
            case = {"lane": lane, "size_mb": mb, "chunk_elems": min(C, S)}
            try:
                if lane in ("onesided", "onesided_wo"):
                    # onesided_wo: window output (calls without out return the
                    # window row of the call: no copy into a caller buffer)
                    kw = {"threads": a.threads} if a.threads else {}
                    wo = lane == "onesided_wo"
                    ar = OneSidedAllreduce(S, max_chunk_size=min(C, S), device=dev, window_output=wo, **kw)
                    # exactness once: integer data, sum in any order is exact
                    y = torch.full((S,), float(rank + 1), device=dev)
                    o = ar(y)
                    torch.cuda.synchronize()
                    case["exact"] = bool((o.data == world * (world + 1) / 2).all()) and bool((o.count == world).all())
                    case["ms"] = _time(lambda: ar(x, out=None if wo else out), a.warmup, a.steps)
                    case["info"] = {k: v for k, v in ar.info().items() if k != "stats"}
                    case["error"] = ar.error()
                    ar.retire()
                    torch.cuda.synchronize()
                    dist.barrier()
                elif lane == "ipc_direct":
                    # the same ipc lane, its rounds launched straight on the
                    # caller's stream (device round ids, ThresholdAllreduce.capturable())
                    ar = ThresholdAllreduce(S, max_chunk_size=min(C, S), device=dev, data_plane="ipc")
                    ar.use_lane(a.ipc_lane)
                    torch.cuda.synchronize()
                    cap = ar.capturable()
                    case["lane"] = a.ipc_lane + "_direct"
                    y = torch.full((S,), float(rank + 1), device=dev)
                    o = cap(y, out=torch.empty_like(y))
                    torch.cuda.synchronize()
                    case["exact"] = bool((o.data == world * (world + 1) / 2).all())
                    case["ms"] = _time(lambda: cap(x, out=out), a.warmup, a.steps)
                    case["error"] = ar.ipc_error()
                    torch.cuda.synchronize()
                    dist.barrier()
                    cap.close()
                else:
                    # the engine path: async rounds (comm stream, event
                    # hand-offs) or, "ipc_sync", synchronous calls (the round
                    # runs on the caller's stream)
                    sync_call = lane == "ipc_sync"
                    ar = ThresholdAllreduce(S, max_chunk_size=min(C, S), device=dev, data_plane="ipc")
                    ar.use_lane(a.ipc_lane)
                    case["lane"] = a.ipc_lane + ("_sync" if sync_call else "")
                    y = torch.full((S,), float(rank + 1), device=dev)
                    o = ar(y)
                    torch.cuda.synchronize()
                    case["exact"] = bool((o.data == world * (world + 1) / 2).all()) and bool((o.count == world).all())
                    case["ms"] = _time(lambda: ar(x, out=out, async_op=not sync_call), a.warmup, a.steps)
                    case["error"] = ar.ipc_error()
                case["algbw_GBps"] = round(S * 4 / (case["ms"] * 1e-3) / 1e9, 2)
            except Exception as e:  # noqa: BLE001 - recorded, the next case still runs
                case["exception"] = f"{type(e).__name__}: {e}"[:300]
            res["cases"].append(case)
            torch.cuda.synchronize()
            dist.barrier()
            del ar
            print(f"rank {rank}: {json.dumps(case)[:300]}", file=sys.stderr, flush=True)
    if a.straggler:
        import bench as B  # noqa: E402  (repo root bench.py)

        res["cfg4"] = B.run_cfg4(world, rank, dev, dist.barrier, a.cfg4_mb, a.delay_ms, a.cfg4_rounds)
    with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
