"""Probe of exact rounds on the one-sided lane at an arbitrary geometry
(torch.distributed.run, ranks sharing the card): per-call ms, verdict and
lane stats, first through OneSidedAllreduce itself, then through
ThresholdAllreduce.use_lane("onesided").  Prints one JSON line per phase."""
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
    ap.add_argument("--size", type=int, default=41_755_624)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=6)
    ap.add_argument("--timeout-s", type=float, default=5.0)
    ap.add_argument("--which", default="direct,engine")
    ap.add_argument("--dp-steps", type=int, default=0, help="then: config 5's MLP DP-SGD step on the lane")
    ap.add_argument("--blocks", default="5,20", help="then: DP steps in blocks without a sync inside")
    ap.add_argument("--cu-keep", type=int, default=6, help="DP lane: CUs kept of every 8 (0: no mask)")
    ap.add_argument("--keep", action="store_true", help="keep the earlier lanes alive (no teardown before the DP lane)")
    ap.add_argument("--gemm", type=int, default=0, help="rank r runs r*GEMM 256x4096x8192 bf16 before each call")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.onesided import OneSidedAllreduce

    x = torch.full((a.size,), float(rank + 1), device=dev)
    ga = torch.randn(256, 4096, device=dev, dtype=torch.bfloat16)
    gb = torch.randn(4096, 8192, device=dev, dtype=torch.bfloat16)
    want = float(world * (world + 1) // 2)
    kept = []
    for which in [w for w in a.which.split(",") if w and w != "none"]:
        if which == "direct":
            ar = OneSidedAllreduce(a.size, max_chunk_size=a.chunk, device=dev, max_lag=1, timeout_s=a.timeout_s)
            call = lambda: ar(x)  # noqa: E731
            os_ = ar
        else:
            ar = ThresholdAllreduce(a.size, max_chunk_size=a.chunk, device=dev, data_plane="ipc")
            ar.use_lane("onesided")
            call = lambda: ar(x)  # noqa: E731
            os_ = ar._exact_os
        rows = []
        for i in range(a.calls):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.gemm * rank):
                ga2 = ga @ gb  # noqa: F841 - another process's compute kernels while the lane waits
            o = call()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            st = o.status if hasattr(o, "status") else {}
            ok = bool((o.data == want).all())
            rows.append({"ms": round(ms, 3), "ok": ok, "reason": st.get("reason"), "round": st.get("round")})
            print(json.dumps({"rank": rank, "which": which, "call": i, **rows[-1]}), flush=True)
        print(json.dumps({"rank": rank, "which": which, "info": os_.info(), "stats": os_.stats(),
                          "error": os_.error()}), flush=True)
        if a.keep:
            kept.append(ar)
        del ar, os_, call, o
        dist.barrier()
    if a.dp_steps:
        from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
        from akka_allreduce_amd.parallel.dp import GradientBucket

        torch.manual_seed(0)
        model = MLP(4096, 8192, 1000).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=a.chunk, device=dev, data_plane="ipc",
                                onesided_options={"timeout_s": a.timeout_s, "cu_keep": a.cu_keep})
        ar.use_lane("onesided")
        ar._exact_os.lane  # noqa: B018 - mapped
        gen = torch.Generator(device=dev).manual_seed(1000 + rank)
        xb, yb = synthetic_batch(256, 4096, 1000, device=dev, generator=gen)
        for i in range(a.dp_steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            loss = dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False)
            torch.cuda.synchronize()
            print(json.dumps({"rank": rank, "dp_step": i, "ms": round((time.perf_counter() - t0) * 1e3, 3),
                              "loss": float(loss), "stats": {k: v for k, v in ar._exact_os.stats().items() if v}}),
                  flush=True)
        for block in [int(b) for b in a.blocks.split(",") if b]:  # config 5's timed() shape: no sync inside a block
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for i in range(block):
                loss = dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False)
            torch.cuda.synchronize()
            print(json.dumps({"rank": rank, "dp_block": block, "ms": round((time.perf_counter() - t0) * 1e3, 3),
                              "stats": {k: v for k, v in ar._exact_os.stats().items()
                                        if k in ("timeouts", "complete_forced", "reduce_forced", "rounds")}}),
                  flush=True)
        print(json.dumps({"rank": rank, "dp_error": ar._exact_os.error()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
