"""Rank program for the one-sided threshold lane tests (tests/test_onesided_cpu.py
on CPU processes over shared memory, tests/test_onesided_gpu.py with every rank
on the box's one GPU).  Run under torch.distributed.run; writes rank<i>.json.

Modes:
  exact      thresholds 1: every round is the fp32 sum in ascending source
             order (bitwise), counts N, round ids 0, 1, 2, ...
  straggler  rank `--straggler` sleeps `--delay-ms` before each call of the
             second phase.  Every rank contributes 2^rank, so each output
             chunk encodes its contributor set: value = sum of 2^s over the
             set and popcount(value) must equal the chunk's count.  Records
             per-call times and round ids of both phases (no straggler /
             straggler) and the lane's stats; `--kill-after K` makes the
             straggler exit abruptly after K calls of the second phase.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def check_sets(o, world, me, dtype, detail=None):
    """Every chunk: value encodes a contributor set whose size is the count.
    `detail` (a list) collects the first few bad chunks, for the report."""
    g = o.geometry
    data = o.data.float().cpu()
    counts = o.counts_per_chunk.cpu()
    bad = 0
    own_has_me = True

    def note(p, k, seg, c):
        if detail is not None and len(detail) < 8:
            vals = torch.unique(seg)
            detail.append({"round": o.iteration, "block": p, "chunk": k, "count": c, "values": vals[:6].tolist(),
                           "n_values": int(vals.numel()), "first_bad": int((seg != seg[0]).nonzero()[0]) if
                           vals.numel() > 1 else -1, "len": int(seg.numel()), "reason": o.status["reason"]})
    for p in range(world):
        for k in range(g.num_chunks(p)):
            s, e = g.chunk_range(p, k)
            if e <= s:
                continue
            seg = data[s:e]
            v = float(seg[0])
            c = int(counts[p, k])
            if not bool((seg == v).all()):
                bad += 1
                note(p, k, seg, c)
                continue
            iv = int(v)
            if float(iv) != v or iv < 0 or iv >= (1 << world) or bin(iv).count("1") != c:
                bad += 1
                note(p, k, seg, c)
            # my own chunk, when it is part of my output (it may be left out:
            # the round can complete before it is reduced, like the reference's
            # completion before the self-delivered ReduceBlock), includes my copy
            if p == me and c > 0 and not (iv >> me) & 1:
                own_has_me = False
    return bad, own_has_me


def bit_share(o, bit):
    """(chunks whose contributor set includes rank ``bit``, chunks): a rank
    whose rounds waited for ``bit``'s copies would have it in every chunk."""
    g = o.geometry
    data, n, hit = o.data.float().cpu(), 0, 0
    for p in range(g.workerNum):
        for k in range(g.num_chunks(p)):
            s, e = g.chunk_range(p, k)
            if e > s:
                n += 1
                hit += (int(float(data[s])) >> bit) & 1
    return hit, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="exact", choices=["exact", "straggler", "chaos", "dead"])
    ap.add_argument("--timeline", action="store_true", help="exact: AKKA_OS_TIMELINE=1, check the stamps")
    ap.add_argument("--async-op", action="store_true", help="exact: async rounds (side stream), wait() then read")
    ap.add_argument("--jitter-ms", type=float, default=2.0, help="chaos: every call waits U(0, jitter) first")
    ap.add_argument("--seed", type=int, default=0, help="chaos: seed offset of the ranks' jitter streams")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--size", type=int, default=1 << 16)
    ap.add_argument("--chunk", type=int, default=1 << 12)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--th", type=float, default=0.75)
    ap.add_argument("--max-lag", type=int, default=1)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--straggler", type=int, default=-1)
    ap.add_argument("--delay-ms", type=float, default=50.0)
    ap.add_argument("--kill-after", type=int, default=-1)
    ap.add_argument("--compute-ms", type=float, default=0.0, help="every rank 'computes' this long before a call")
    ap.add_argument("--part-bytes", type=int, default=0, help="0: the lane default part size")
    ap.add_argument("--timeout-s", type=float, default=30.0)
    ap.add_argument("--handoff", default="lite", choices=["lite", "fenced"])
    ap.add_argument("--window-output", action="store_true", help="exact: calls without out return window rows")
    ap.add_argument("--out-dir", required=True)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    if a.device == "cuda":
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    dtype = torch.float32 if a.dtype == "float32" else torch.bfloat16
    from akka_allreduce_amd.parallel.onesided import OneSidedAllreduce

    if a.timeline:
        os.environ["AKKA_OS_TIMELINE"] = "1"  # read by each call's launch
    th = 1.0 if a.mode in ("exact", "dead") else a.th
    ar = OneSidedAllreduce(a.size, max_chunk_size=a.chunk, dtype=dtype, th_reduce=th, th_complete=th,
                           max_lag=a.max_lag, device=dev, rows=a.rows, part_bytes=a.part_bytes,
                           timeout_s=a.timeout_s, handoff=a.handoff, window_output=a.window_output)
    res = {"rank": rank, "info": ar.info()}

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    if a.mode == "exact":
        res["exact"], res["rounds"] = [], []
        for r in range(a.rounds):
            x = torch.randn(a.size, generator=torch.Generator().manual_seed(1000 * rank + r)).to(dtype)
            xd = x.to(dev)
            o = ar(xd, async_op=a.async_op)
            if a.async_op:
                o.wait()
            sync()
            want = None
            for s in range(world):
                y = torch.randn(a.size, generator=torch.Generator().manual_seed(1000 * s + r)).to(dtype).float()
                want = y if want is None else want + y
            ok = torch.equal(o.data.cpu(), want.to(dtype)) and bool((o.count.cpu() == world).all())
            res["exact"].append(bool(ok))
            res["rounds"].append(o.iteration)
            if ar.window_output:  # the output IS the window row of this call's id
                res.setdefault("in_window", []).append(
                    o.data.data_ptr() == ar._rows[r % len(ar._rows)].data_ptr())
        if a.timeline:
            tl = ar.lane.timeline()
            g = ar.info()["role_wgs"]
            grid = 1 + g["push"] + ar.geometry.num_chunks(rank) + g["reduce"] + 1 + g["copy"]
            w = [tl[i:i + 3] for i in range(0, len(tl), 3)][:grid]
            res["timeline"] = {"words": len(tl), "grid": grid,
                               "ordered": all(0 < t[0] <= t[1] <= t[2] for t in w),
                               "span_ticks": (max(t[2] for t in w) - min(t[0] for t in w)) if w else 0}
    elif a.mode == "dead":
        # exact thresholds; rank N-1 serves `kill_after` rounds, then vanishes
        # without retiring (its window stays mapped); the survivors learn it
        # out of band (the master's WorkerTerminated, M:46-52) and mark it
        # dead: later rounds complete over the live ranks, the dead rank's
        # block 0 with count 0, every live block the exact live sum
        victim, k = world - 1, max(1, a.kill_after)
        x = torch.full((a.size,), float(1 << rank), dtype=dtype, device=dev)
        out = torch.empty_like(x)
        res["dead"] = {"before": [], "after": [], "reasons": []}
        for i in range(k):
            o = ar(x, out=out)
            sync()
            res["dead"]["before"].append(o.iteration)
        if rank == victim:
            dist.barrier()  # the survivors are past round k-1 too
            with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
                json.dump(res, f)
            os._exit(0)
        dist.barrier()
        ar.mark_dead(victim)
        live = sum(1 << q for q in range(world) if q != victim)
        g = ar.geometry
        bad = 0
        for i in range(a.rounds):
            o = ar(x, out=out)
            sync()
            data, cnt = o.data.float().cpu(), o.counts_per_chunk.cpu()
            for p in range(world):
                for kk in range(g.num_chunks(p)):
                    s0, e0 = g.chunk_range(p, kk)
                    if e0 <= s0:
                        continue
                    want_v, want_c = (0.0, 0) if p == victim else (float(live), world - 1)
                    if not (bool((data[s0:e0] == want_v).all()) and int(cnt[p, kk]) == want_c):
                        bad += 1
            res["dead"]["after"].append(o.iteration)
            res["dead"]["reasons"].append(o.status["reason"])
        res["dead"]["bad_chunks"] = bad
        res["error"] = ar.error()
        res["stats"] = ar.stats()
        with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
        os._exit(0)  # a peer is gone: no collective teardown
    elif a.mode == "chaos":
        # every rank waits a random time before each call (its own seeded
        # stream): arrival orders, lags, catch-ups and overwrite conflicts
        # all vary from round to round; every output chunk is checked
        import random

        rng = random.Random(1234 + rank + 1000 * a.seed)
        x = torch.full((a.size,), float(1 << rank), dtype=dtype, device=dev)
        out = torch.empty_like(x)
        bad, detail, rounds, reasons, last, partial = 0, [], [], [], -1, 0
        while last < a.rounds - 1:
            time.sleep(rng.uniform(0.0, a.jitter_ms) / 1e3)
            o = ar(x) if a.window_output else ar(x, out=out)
            sync()
            b, _ = check_sets(o, world, rank, dtype, detail)
            bad += b
            cnt, g = o.counts_per_chunk.cpu(), o.geometry  # a chunk short of N contributors?
            partial += int(any(int(cnt[p, k]) != world for p in range(world) for k in range(g.num_chunks(p))
                               if g.chunk_range(p, k)[1] > g.chunk_range(p, k)[0]))
            last = o.iteration
            rounds.append(last)
            reasons.append(o.status["reason"])
        res["chaos"] = {"rounds": rounds, "bad_chunks": bad, "bad_detail": detail, "reasons": reasons,
                        "calls_with_partial_chunks": partial,
                        "stats": ar.stats()}
        ar.retire()
        sync()
    else:
        x = torch.full((a.size,), float(1 << rank), dtype=dtype, device=dev)
        out = torch.empty_like(x)
        # A phase ends at a common ROUND, not a call count: with thresholds < 1
        # a rank can complete rounds without a slow peer and skip ahead by
        # catch-up, so call counts differ between ranks (the reference's
        # master ends the job at maxRound the same way, M:58-63).
        for pi, phase in enumerate(("no_straggler", "straggler")):
            times, rounds, bad, own_ok, reasons, detail = [], [], 0, True, [], []
            with_s, nchunks = 0, 0
            target, last, c = (pi + 1) * a.rounds - 1, -1 if pi == 0 else res["no_straggler"]["rounds"][-1], 0
            while last < target:
                c += 1
                if phase == "straggler" and rank == a.straggler:
                    if c == a.kill_after:
                        sync()
                        res["killed_after"] = c
                        with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
                            json.dump(res, f)
                        os._exit(0)  # abrupt: no retire, no teardown
                    time.sleep(a.delay_ms / 1e3)
                elif a.compute_ms:
                    time.sleep(a.compute_ms / 1e3)
                t0 = time.perf_counter()
                o = ar(x, out=out)
                sync()
                times.append((time.perf_counter() - t0) * 1e3)
                b, mine = check_sets(o, world, rank, dtype, detail)
                bad += b
                own_ok &= mine
                if a.straggler >= 0:
                    h, n = bit_share(o, a.straggler)
                    with_s, nchunks = with_s + h, nchunks + n
                last = o.iteration
                rounds.append(last)
                reasons.append(o.status["reason"])
            res[phase] = {"ms": times, "rounds": rounds, "bad_chunks": bad, "own_block_has_me": own_ok,
                          "reasons": reasons, "stats": ar.stats(), "bad_detail": detail,
                          "chunks_with_straggler": with_s, "chunks": nchunks}
        ar.retire()
        sync()
    res["error"] = ar.error()
    res["stats"] = ar.stats()
    if a.mode == "exact" and ar.window_output and not a.async_op:
        # a window row outlives the allreduce object: the tensor keeps the
        # lane (and its window memory) alive -- read it after every rank
        # dropped its object and the lanes' teardown would have freed it
        import gc
        import weakref

        keep, want_last = o.data, want.to(dtype)
        lane_ref = weakref.ref(ar.lane)
        del o, ar
        gc.collect()
        dist.barrier()
        res["kept_row_alive"] = lane_ref() is not None
        res["kept_row_exact"] = bool(torch.equal(keep.cpu(), want_last))
        del keep
        gc.collect()
        res["row_dropped_frees_lane"] = lane_ref() is None
    with open(os.path.join(a.out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    sys.stdout.flush()
    if a.kill_after < 0:
        dist.barrier()
        dist.destroy_process_group()
    else:
        os._exit(0)  # a peer is gone: no collective teardown


if __name__ == "__main__":
    main()
