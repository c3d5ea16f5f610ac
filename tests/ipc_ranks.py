"""Rank program for tests/test_ipc_gpu.py (run under torch.distributed.run):
every rank of the job drives the SAME GPU (a 1-GPU box), with the ipc-only data
plane -- windows in one process's HBM mapped into the others through IPC
handles, so the push / reduce / pull kernels, their round-id flags and the
cross-process hand-offs run for real (cross-XCD, not cross-xGMI).  Prints one
JSON line per rank."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def expected(S, world, r, dtype, g_seed):
    acc = None
    for src in range(world):
        x = torch.randn(S, generator=torch.Generator().manual_seed(g_seed * 1000 + src * 7 + r), dtype=torch.float32)
        x = x.to(dtype).float()
        acc = x if acc is None else acc + x  # ascending source rank, fp32 (the kernel's order)
    return acc.to(dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--skip-rank", type=int, default=-1, help="this rank runs only round 0 (a missing peer)")
    ap.add_argument("--late-rank", type=int, default=-1, help="this rank sleeps --late-s before round 1")
    ap.add_argument("--late-s", type=float, default=0.0)
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--time-mode", default="", choices=["", "pull", "bcast", "fused", "fused_bcast"],
                    help="phase-2 mode of the timed rounds (--rounds 0 times without checking)")
    ap.add_argument("--chunk", type=int, default=0, help="max chunk size (elements; default size / 16)")
    ap.add_argument("--time-async", action="store_true", help="timed rounds with async_op=True")
    ap.add_argument("--pre-size", type=int, default=0, help="run 5 rounds of another fp32 engine of this size first")
    ap.add_argument("--pre-rounds", type=int, default=5, help="rounds of the --pre-size engine")
    ap.add_argument("--pre-del", action="store_true", help="delete the --pre-size engine before the timed one")
    ap.add_argument("--mode", default="pull", choices=["pull", "bcast", "alternate", "fused", "fused_bcast", "rotate"])
    ap.add_argument("--out-dir", default="", help="write rank<i>.json there (stdout lines of ranks interleave)")
    ap.add_argument("--lane-seq", default="",
                    help="comma list of lane names (ThresholdAllreduce.LANES): use_lane(name) before round r "
                         "(cycled); records the lane's round id after each round")
    ap.add_argument("--poison", action="store_true",
                    help="round 0 runs on a fresh stream whose only free block is still being written by a "
                         "pending spin + fill: the round's output/counts are carved from it")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dtype = torch.float32 if a.dtype == "float32" else torch.bfloat16
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    pre = None
    if a.pre_size:  # another engine in the process first (bench.py's headline before its extras)
        pre = ThresholdAllreduce(a.pre_size, max_chunk_size=max(1, a.pre_size // 64), device=dev, data_plane="ipc")
        px = torch.randn(a.pre_size, device=dev)
        for _ in range(a.pre_rounds):
            pre(px, async_op=True).wait()
        torch.cuda.synchronize()
        if a.pre_del:
            dist.barrier()  # every rank's pre rounds drained before any window goes
            del pre, px
            import gc

            gc.collect()
            pre = None
    ar = ThresholdAllreduce(a.size, max_chunk_size=a.chunk or max(1, a.size // 16), dtype=dtype, device=dev,
                            data_plane="ipc")
    res = {"rank": rank, "exact": [], "lane": ar.state()["link"]["lane"],
           "ipc_open_s": getattr(ar, "ipc_open_s", None)}
    for r in range(a.rounds):
        if r > 0 and rank == a.skip_rank:
            break
        if r == 1 and rank == a.late_rank:
            import time

            time.sleep(a.late_s)  # arrives after the peers' waits timed out
        if a.lane_seq:
            seq = a.lane_seq.split(",")
            ar.use_lane(seq[r % len(seq)])
        elif a.mode != "pull":
            variants = [("pull", False), ("bcast", False), ("pull", True), ("bcast", True)]
            mode, fused = {"bcast": ("bcast", False), "fused": ("pull", True), "fused_bcast": ("bcast", True),
                           "alternate": variants[r % 2], "rotate": variants[r % 4]}[a.mode]
            ar.set_ipc_mode(mode, fused)
        x = torch.randn(a.size, generator=torch.Generator().manual_seed(5 * 1000 + rank * 7 + r),
                        dtype=torch.float32).to(dtype).to(dev)
        if a.poison and r == 0:
            torch.cuda.synchronize()
            side = torch.cuda.Stream()
            with torch.cuda.stream(side):
                junk = torch.empty((a.size * x.element_size() + 4096) // 4, dtype=torch.int32, device=dev)
                torch.cuda._sleep(200_000_000)  # the fill below lands ~0.1 s later in this stream's order
                junk.fill_(-7)
                lo, hi = junk.data_ptr(), junk.data_ptr() + junk.numel() * 4
                del junk  # free at once for this stream's next allocations
                o = ar(x)
                res["poison_in_block"] = lo <= o.counts_per_chunk.data_ptr() < hi
            side.synchronize()
            res["poison_counts_ok"] = bool((o.counts_per_chunk == world).all())
        else:
            o = ar(x)
        torch.cuda.synchronize()
        want = expected(a.size, world, r, dtype, 5)
        res["exact"].append(bool(torch.equal(o.data.cpu(), want)) and bool((o.count.cpu() == world).all()))
        res.setdefault("counts_all_zero", []).append(bool((o.counts_per_chunk.cpu() == 0).all()))
        if a.lane_seq:  # the lane's round id, host or device resident (synchronises)
            res.setdefault("lane_round", []).append(int(ar.worker._core.ipc_current_round()))
    res["ipc_error"] = ar.ipc_error()
    if ((a.skip_rank >= 0 and rank != a.skip_rank) or a.late_rank >= 0) and res["ipc_error"]:
        # the next round on this lane refuses to run (like an RCCL async error)
        try:
            ar(torch.zeros(a.size, device=dev, dtype=dtype))
            res["next_round_raised"] = False
        except Exception as e:  # noqa: BLE001
            res["next_round_raised"] = "timed out" in str(e)
    st = ar.state()["link"]
    res["ipc_rounds"] = st["ipc_rounds"]
    res["ipc"] = st.get("ipc")
    if a.time and a.skip_rank < 0:
        if a.time_mode:
            ar.set_ipc_mode(*{"pull": ("pull", False), "bcast": ("bcast", False), "fused": ("pull", True),
                              "fused_bcast": ("bcast", True)}[a.time_mode])
        x = torch.randn(a.size, device=dev).to(dtype)
        out = torch.empty_like(x)
        o = None
        for _ in range(3):
            o = ar(x, out=out, async_op=a.time_async)
        o.wait()
        torch.cuda.synchronize()
        dist.barrier()
        import time

        t0 = time.perf_counter()
        k = 10
        for _ in range(k):
            o = ar(x, out=out, async_op=a.time_async)
        o.wait()
        torch.cuda.synchronize()
        dist.barrier()
        res["ms_per_round"] = (time.perf_counter() - t0) / k * 1e3
    if a.out_dir:
        with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
    else:
        print(json.dumps(res), flush=True)
    # every rank's kernels have drained (ipc_error synchronised) before any
    # window is released
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
