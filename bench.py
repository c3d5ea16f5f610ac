#!/usr/bin/env python3
"""Headline benchmark: allreduce algbw (GB/s) on a 256 MB fp32 buffer, 1/2/4/8 MI355X.

Metric and config come from BASELINE.json.  One rank per GPU; for N>1 the
driver launches this file under ``torch.distributed.run`` (RANK/LOCAL_RANK/
WORLD_SIZE/MASTER_* in the env).  Each timed step is one full threshold-
allreduce round through the native engine: scatter of every chunk to its
owner over RCCL/xGMI, the gfx950 chunk-reduce kernel, broadcast of the reduced
chunks, counts exchange, and hand-off of a fresh output tensor.  Data is
synthetic random fp32 (no dataset involved).  Exact thresholds (1.0/1.0/1.0)
as in BASELINE config 2.

algbw = buffer bytes / seconds per round; busbw = algbw * 2(N-1)/N.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_METRIC = "allreduce algbw (GB/s) on 256 MB fp32 buffer at 1/2/4/8 MI355X"
XGMI_LINK_GBPS = 153.0  # per-link figure used for the analytic bound, not measured here


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size-mb", type=float, default=256.0, help="buffer size in MiB (256 MB headline)")
    p.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    p.add_argument("--chunk-mb", type=float, default=4.0, help="maxChunkSize in MiB (BASELINE config 2: 4 MB)")
    p.add_argument("--max-lag", type=int, default=2)
    p.add_argument("--bcast-lag", type=int, default=2)
    p.add_argument("--th-reduce", type=float, default=1.0)
    p.add_argument("--th-complete", type=float, default=1.0)
    p.add_argument("--compare-rccl", choices=["auto", "on", "off"], default="auto",
                   help="also time torch.distributed all_reduce (RCCL) on the same buffer after the timed "
                        "region -- auto: on for N>1")
    p.add_argument("--no-check", action="store_true")
    p.add_argument("--extras", choices=["auto", "on", "off"], default="auto",
                   help="after the headline, also time BASELINE config 3 (bf16 1 GiB) and config 5 (MLP DP-SGD) "
                        "-- auto: only for the default headline invocation")
    p.add_argument("--watchdog-s", type=float, default=900.0,
                   help="dump stacks and exit if the run is not done after this many seconds (0: off)")
    p.add_argument("--phase-deadline-s", type=float, default=180.0,
                   help="per-phase deadline (init, rccl_init, warmup, timed, ...): on expiry rank 0 prints one JSON "
                        "line with failed_phase and the RCCL debug tail, and every rank exits non-zero")
    p.add_argument("--preflight-deadline-s", type=float, default=120.0,
                   help="deadline of the exact preflight round run before timing at N>1")
    p.add_argument("--preflight", choices=["auto", "on"], default="auto",
                   help="auto: preflight round only at N>1")
    p.add_argument("--pg-timeout-s", type=float, default=300.0, help="host (gloo) process group timeout")
    p.add_argument("--extras-only", default="", help="comma list of extra configs to run (cfg1,cfg3,cfg4,cfg5)")
    p.add_argument("--cfg4-size-mb", type=float, default=64.0, help="config 4 buffer (MiB)")
    p.add_argument("--cfg4-delay-ms", type=float, default=50.0, help="config 4 straggler delay per round")
    p.add_argument("--cfg4-rounds", type=int, default=64,
                   help="rounds per phase of config 4 (steady state: far more rounds than any buffering)")
    p.add_argument("--cfg4-transport", choices=["onesided", "reactive"], default="onesided",
                   help="config 4 data path: onesided (stores into mapped peer windows, no send ever waits) or "
                        "reactive (RCCL pair communicators, two-sided)")
    p.add_argument("--link-probe", choices=["on", "off"], default="on",
                   help="N>1: measure every ordered pair's push / pull bandwidth after the headline (untimed)")
    p.add_argument("--link-probe-mib", type=float, default=64.0)
    p.add_argument("--link-probe-deadline-s", type=float, default=120.0)
    p.add_argument("--extras-deadline-s", type=float, default=240.0,
                   help="give up on the extra configs after this many seconds (the headline line is still printed)")
    p.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                   help="cpu: rehearse the multi-rank flow on gloo (CPU tests); numbers are not the metric")
    p.add_argument("--fresh-out", action="store_true", help="allocate a new output tensor every round")
    p.add_argument("--transport", choices=["stream", "reactive"], default="stream",
                   help="stream: symmetric step schedule on one comm stream (default); reactive: per-peer streams + "
                        "pair communicators, event-polled arrivals (straggler-tolerant)")
    p.add_argument("--lane", choices=["auto", "p2p", "collective"], default="auto",
                   help="exact-round lane of the stream transport (stream_link.h): auto = RCCL reduce-scatter + "
                        "all-gather when the buffer splits evenly, else the chunk-pipelined p2p schedule")
    p.add_argument("--lane-select", choices=["on", "off"], default="on",
                   help="with --lane auto at N>1 (stream transport): before the warmup, run one exact round and a "
                        "few timed rounds on each lane and keep the faster exact one (every rank agrees)")
    p.add_argument("--data-plane", choices=["rccl", "ipc", "ipc_p2p"], default="rccl",
                   help="ipc: no RCCL communicator, every exact round on the one-sided xGMI lane; ipc_p2p: the "
                        "p2p schedules over mailboxes in mapped peer memory (with AKKA_SHARE_GPU=1 either rehearses "
                        "the N-rank flow with N processes on one card)")
    p.add_argument("--lane-output", choices=["on", "off"], default="on",
                   help="on: a one-sided lane chosen for the timed rounds returns its window row (no copy into a "
                        "caller buffer; the output of a round is valid until the next round)")
    p.add_argument("--ipc", choices=["on", "off"], default="on",
                   help="lane selection also tries the one-sided xGMI lane (mapped peer windows, ipc_lane.h)")
    p.add_argument("--async-op", choices=["auto", "on", "off"], default="auto",
                   help="async rounds (event hand-off) -- auto: on for N>1 (saves a stream hop per round), off for "
                        "N=1 (local rounds run on the caller's stream, nothing to hop)")
    return p.parse_args()


def _sync() -> None:
    """Device synchronize (no-op for the --device cpu rehearsal)."""
    import torch

    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def timed(step, steps: int, warmup: int, world: int, barrier) -> float:
    """Seconds for `steps` calls of step() (after `warmup`), barrier +
    synchronize on both sides, max over ranks."""
    import torch
    import torch.distributed as dist

    def finish(o):
        if hasattr(o, "wait"):
            o.wait()
        _sync()
        barrier()
        _sync()

    o = None
    for _ in range(warmup):
        o = step()
    finish(o)
    t0 = time.perf_counter()
    for _ in range(steps):
        o = step()
    finish(o)
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


class _Skip(Exception):
    pass


def run_cfg4(world: int, rank: int, dev, barrier, size_mb: float, delay_ms: float, rounds: int) -> dict:
    """BASELINE config 4 on the one-sided lane (transport="onesided",
    csrc/transport/onesided.h): thReduce = thComplete = 0.75, maxLag 1, rank
    N-1 an induced straggler.  Every send is a store into the receiver's
    window, so the fast ranks never wait for the straggler -- in steady state,
    not only until a buffer pool runs out (reference: fire-and-forget sends
    W:227-232 / 259-264, outdated drops W:155-156 / 172-173, thresholds
    SB:9-13 / RB:13-17, catch-up W:100-106).

    Two phases of `rounds` rounds each, each ending at a common ROUND (with
    thresholds < 1 ranks skip rounds by catch-up, so their call counts
    differ): without the straggler, then with rank N-1 sleeping `delay_ms`
    before each call.  Per phase: the fast ranks' median and p90 ms per call
    over the second half (worst fast rank), their mean contributor count, the
    straggler's calls and catch-up skips, drops and forced reduces.

    Then an untimed validation phase (`validation`, straggler still late):
    every rank contributes the constant 2^rank, so every output chunk must be
    one integer whose set bits are its contributors, as many as its count --
    a torn, stale or mixed chunk shows (on a node: the cross-device hand-offs
    of the one-sided lane, checked on the job itself).

    The lane starts with its fast "lite" hand-offs (write-through stores +
    drain).  If the validation finds a bad chunk on any rank, every rank
    switches to the FENCED hand-off (system release / acquire, the HIP memory
    model's own protocol) and runs both phases and the validation again: the
    line then says ``handoff: fenced`` and keeps the lite run under
    ``handoff_fallback`` -- the straggler path stays available whatever the
    link does (reference: AllreduceWorker.scala:170-186)."""
    import torch

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    esize = 4
    S = int(size_mb * (1 << 20)) // esize
    C = max(1, min(S, (4 << 20) // esize))
    ar = ThresholdAllreduce(S, max_chunk_size=C, th_reduce=0.75, th_complete=0.75, max_lag=1, device=dev,
                            transport="onesided")
    run_cfg4.keep = ar  # type: ignore[attr-defined]
    straggler = world - 1
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    x = torch.randn(S, device=dev, generator=g)
    out = torch.empty_like(x)
    res = {"thresholds": [1.0, 0.75, 0.75], "max_lag": 1, "straggler_rank": straggler, "straggler_delay_ms": delay_ms,
           "rounds_per_phase": rounds, "buffer_bytes": S * esize, "chunk_bytes": C * esize, "transport": "onesided",
           "lane": ar.state()["link"]["onesided"]}
    res["lane"].pop("stats", None)
    res.update(cfg4_threshold_needs(world, S, C, 0.75, 0.75, straggler))
    res["handoff"] = ar._os.handoff
    res["handoff_fallback"] = None

    def sync():
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()

    # every rank's setup kernels done before any round starts: on a shared
    # card a peer's waiting round could otherwise hold the SIMDs a late
    # rank's setup kernels need (docs/DESIGN.md §4c, cu_keep)
    sync()
    barrier()
    last = cfg4_phases(ar, res, x, out, world, rank, straggler, delay_ms, rounds, -1, sync)
    res["validation"] = cfg4_validate(ar, world, rank, straggler, delay_ms, last, max(8, rounds // 4), dev)
    last = res["validation"].pop("last_round")
    if not res["validation"]["contributor_sets_consistent"] and ar._os.handoff != "fenced":
        # a torn, stale or mixed chunk on the lite hand-offs (the verdict is
        # the same on every rank: the validation gathers every rank's count)
        lite = {k: res.pop(k) for k in ("no_straggler", "with_straggler", "fast_rank_slowdown", "validation")}
        ar._os.set_handoff("fenced")
        sync()
        barrier()
        last = cfg4_phases(ar, res, x, out, world, rank, straggler, delay_ms, rounds, last, sync)
        res["validation"] = cfg4_validate(ar, world, rank, straggler, delay_ms, last, max(8, rounds // 4), dev)
        res["validation"].pop("last_round")
        res["handoff"] = "fenced"
        res["handoff_fallback"] = {"from": "lite", "reason": "validation found torn / stale / mixed chunks",
                                   "lite": lite}
    ar.retire()  # the job's end: nobody waits for this rank's later rounds
    sync()
    barrier()
    return res


def cfg4_phases(ar, res: dict, x, out, world: int, rank: int, straggler: int, delay_ms: float, rounds: int,
                last: int, sync) -> int:
    """Config 4's two timed phases (run_cfg4), each ending at a common round
    past ``last`` (the same on every rank); fills ``res``, returns this
    rank's last round served."""
    import statistics

    import torch
    import torch.distributed as dist

    base = last + 1
    for pi, key in enumerate(("no_straggler", "with_straggler")):
        target = base + (pi + 1) * rounds - 1
        st0 = ar._os.stats()
        ms, outs, calls = [], [], 0
        while last < target:
            if key == "with_straggler" and rank == straggler:
                time.sleep(delay_ms / 1e3)
            t0 = time.perf_counter()
            o = ar(x, out=out)
            sync()
            ms.append((time.perf_counter() - t0) * 1e3)
            # the call's record is host memory the final kernel wrote: read
            # without another stream synchronisation; counts are resolved
            # after the phase (one device copy per phase, not per call)
            last = o.status_nowait()["round"]
            outs.append(o.counts_per_chunk.sum())
            calls += 1
        nch = float(sum(ar._os.geometry.num_chunks(p) for p in range(world)))
        cnt = [float(v) / max(1.0, nch) for v in torch.stack(outs).cpu().tolist()]  # mean per-chunk count
        st1 = ar._os.stats()
        tail = sorted(ms[len(ms) // 2:])
        mine = {"median_ms": statistics.median(tail), "p90_ms": tail[min(len(tail) - 1, int(0.9 * len(tail)))],
                "calls": calls, "mean_count": sum(cnt) / len(cnt),
                **{k: st1[k] - st0[k] for k in ("skipped_rounds", "scatter_outdated", "gather_outdated",
                                                 "scatter_conflict", "gather_conflict", "reduce_forced",
                                                 "complete_forced", "timeouts")}}
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        fast = [v for i, v in enumerate(allv) if i != straggler]
        res[key] = {
            "fast_rank_median_ms_per_round": round(max(v["median_ms"] for v in fast), 4),
            "fast_rank_p90_ms_per_round": round(max(v["p90_ms"] for v in fast), 4),
            "fast_rank_mean_count": round(sum(v["mean_count"] for v in fast) / len(fast), 4),
            "fast_rank_calls": [v["calls"] for v in fast],
            "straggler_calls": allv[straggler]["calls"],
            "straggler_median_ms_per_call": round(allv[straggler]["median_ms"], 4),
            "catch_up_skipped_rounds": sum(v["skipped_rounds"] for v in allv),
            "outdated_pushes_dropped": sum(v["scatter_outdated"] + v["gather_outdated"] for v in allv),
            "straggler_outdated_pushes_dropped": allv[straggler]["scatter_outdated"] + allv[straggler]["gather_outdated"],
            "conflict_drops": sum(v["scatter_conflict"] + v["gather_conflict"] for v in allv),
            "forced_chunk_reduces": sum(v["reduce_forced"] for v in allv),
            "forced_completions": sum(v["complete_forced"] for v in allv),
            "timeouts": sum(v["timeouts"] for v in allv),
        }
        # the next phase starts past the largest round any rank served
        lasts = [None] * world
        dist.all_gather_object(lasts, last)
        last = max(lasts)
    a, b = res["no_straggler"], res["with_straggler"]
    res["fast_rank_slowdown"] = round(b["fast_rank_median_ms_per_round"] / max(1e-9, a["fast_rank_median_ms_per_round"]),
                                      3)
    return last


def cfg4_validate(ar, world: int, rank: int, straggler: int, delay_ms: float, last: int, rounds: int, dev) -> dict:
    """Config 4's untimed validation rounds (run_cfg4): inputs 2^rank, every
    chunk of every output checked against its contributor count."""
    import torch
    import torch.distributed as dist

    from akka_allreduce_amd.utils.faults import env_bad_handoff

    os_ = ar._os
    g = os_.geometry
    inject = env_bad_handoff(rank, os_.handoff)  # fault injection: one torn chunk per call
    S = ar.data_size
    x = torch.full((S,), float(1 << rank), device=dev)
    out = torch.empty_like(x)
    bad, chunks, calls, first_bad = 0, 0, 0, None
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)  # x is written before any peer's round can wait on this rank
    lasts = [None] * world
    dist.all_gather_object(lasts, last)
    target = max(lasts) + rounds  # a common round, like the timed phases
    while last < target:
        if rank == straggler:
            time.sleep(delay_ms / 1e3)
        o = ar(x, out=out)
        data = o.data.float().cpu()
        counts = o.counts_per_chunk.cpu()
        last = o.status_nowait()["round"]
        calls += 1
        for p in range(world):
            for k in range(g.num_chunks(p)):
                s0, e0 = g.chunk_range(p, k)
                if e0 <= s0:
                    continue
                chunks += 1
                seg = data[s0:e0]
                v, c = float(seg[0]), int(counts[p, k])
                iv = int(v)
                ok = bool((seg == v).all()) and float(iv) == v and 0 <= iv < (1 << world) and bin(iv).count("1") == c
                if inject and p == 0 and k == 0:
                    ok = False
                if not ok:
                    bad += 1
                    if first_bad is None:
                        first_bad = {"round": last, "block": p, "chunk": k, "count": c, "value": v}
    mine = {"bad": bad, "chunks": chunks, "calls": calls, "first_bad": first_bad, "last": last}
    allv = [None] * world
    dist.all_gather_object(allv, mine)
    return {"rounds": rounds, "handoff": os_.handoff, "last_round": max(v["last"] for v in allv),
            "calls": [v["calls"] for v in allv], "chunks_checked": sum(v["chunks"] for v in allv),
            "bad_chunks": sum(v["bad"] for v in allv),
            "first_bad": next((dict(v["first_bad"], rank=i) for i, v in enumerate(allv) if v["first_bad"]), None),
            "contributor_sets_consistent": all(v["bad"] == 0 for v in allv)}


def cfg4_threshold_needs(world: int, S: int, C: int, th_reduce: float, th_complete: float, straggler: int) -> dict:
    """What config 4's thresholds demand at this N (float32 products, like
    the reference, SB:9 / RB:13-17).  ``straggler_block_required``: the
    completion threshold cannot be met by the other ranks' chunks alone, so
    every round waits for (or is forced without) the straggler's block --
    at N=2 with 16 chunks, floor(0.75*16) = 12 > 16 - 8."""
    import numpy as np

    from akka_allreduce_amd.data import Geometry

    g = Geometry(S, world, C)
    total = sum(g.num_chunks(p) for p in range(world))
    need_c = int(np.floor(np.float32(th_complete) * np.float32(total)))
    need_r = int(np.floor(np.float32(th_reduce) * np.float32(world)))
    strag = g.num_chunks(straggler)
    return {"total_chunks": total, "need_complete_chunks": need_c, "need_reduce_copies": need_r,
            "straggler_chunks": strag,
            "straggler_block_required": need_c > total - strag,
            "straggler_copy_required": need_r > world - 1}


def run_cfg4_reactive(world: int, rank: int, dev, barrier, size_mb: float, delay_ms: float, rounds: int,
                      data_plane: str = "rccl") -> dict:
    """BASELINE config 4: threshold allreduce at thReduce = thComplete = 0.75,
    maxLag 1, with rank N-1 an induced straggler (sleeps ``delay_ms`` before
    each round), on the straggler-tolerant reactive transport (one pair
    communicator + stream per peer, reactive_link.h).  Reports the fast ranks'
    time per round with and without the straggler (max over the fast ranks),
    the mean contributor count they saw, and the forced (catch-up) rounds.
    Reference: thresholds SB:9-13 / RB:13-17, catch-up W:100-106, pacing M:58.
    With N < 4, 0.75 of the chunks cannot complete without the straggler's
    block, so the fast ranks wait for it -- the reported times show that."""
    import torch
    import torch.distributed as dist

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    esize = 4
    S = int(size_mb * (1 << 20)) // esize
    C = max(1, min(S, (4 << 20) // esize))
    ar = ThresholdAllreduce(S, max_chunk_size=C, th_reduce=0.75, th_complete=0.75, max_lag=1, device=dev,
                            transport="reactive", data_plane=data_plane)
    run_cfg4_reactive.keep = ar  # type: ignore[attr-defined]
    straggler = world - 1
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    x = torch.randn(S, device=dev, generator=g)
    res = {"thresholds": [1.0, 0.75, 0.75], "max_lag": 1, "straggler_rank": straggler,
           "straggler_delay_ms": delay_ms, "rounds": rounds, "buffer_bytes": S * esize, "transport": "reactive"}

    def phase(delay_s: float):
        ar.fault_delay_s = delay_s if rank == straggler else 0.0
        outs = []
        t0 = time.perf_counter()
        for _ in range(rounds):
            outs.append(ar(x))
        # every round's output is ready on the caller's stream (the round's done
        # point is waited for there); a device-wide synchronize would also wait
        # for the transfers still parked on the straggler's pair stream -- the
        # very wait this config shows the fast ranks do not need
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()
        dt = time.perf_counter() - t0
        cnt = [float(o.count.float().mean()) for o in outs]
        ar.fault_delay_s = 0.0
        ar.drain()  # every transfer of this rank done before the blocking collectives
        _sync()
        barrier()
        return dt, sum(cnt) / len(cnt)

    phase(0.0)  # warm-up: pair connections, send-slot pool
    for key, delay_s in (("no_straggler", 0.0), ("with_straggler", delay_ms / 1e3)):
        forced0 = ar.state()["stats"]["rounds_forced"]
        dt, mean_count = phase(delay_s)
        forced = ar.state()["stats"]["rounds_forced"] - forced0
        t = torch.tensor([dt / rounds * 1e3, mean_count, float(forced)], dtype=torch.float64)
        allv = [torch.zeros_like(t) for _ in range(world)] if world > 1 else [t]
        if world > 1:
            dist.all_gather(allv, t)
        fast = [v for i, v in enumerate(allv) if i != straggler] or allv
        res[f"fast_rank_ms_per_round_{key}"] = round(max(float(v[0]) for v in fast), 3)
        res[f"straggler_ms_per_round_{key}"] = round(float(allv[straggler][0]), 3)
        res[f"fast_rank_mean_count_{key}"] = round(sum(float(v[1]) for v in fast) / len(fast), 4)
        res[f"forced_rounds_{key}"] = int(sum(float(v[2]) for v in allv))
    return res


def run_cfg1(rounds: int = 300, gpu: bool = False) -> dict:
    """BASELINE config 1, the reference's README demo: a master and 2 worker
    PROCESSES (the CLI, as `sbt runMain ...` in the reference) over loopback
    TCP, dataSize 10, maxChunkSize 2, maxLag 1, CPU data plane.  Run twice:
    the demo's thresholds (1 / 1 / 0.8, M:98-107) and exact thresholds with
    the sink's assertMultiple check (W:337-340).  Reports rounds per second
    and the sink's own MB/s figure (W:329-342) over the last checkpoint
    interval of each worker.  ``gpu``: a third run with the workers on this
    GPU and their data plane on the one-sided lane (master hosts the window
    rendezvous, paces with thAllreduce), exact thresholds + assertMultiple."""
    import re
    import socket
    import subprocess
    import tempfile

    from akka_allreduce_amd._native_loader import load as _load_native

    wd = _load_native()
    base = [sys.executable, "-m", "akka_allreduce_amd", "--log-level", "WARNING"]
    cp = max(1, rounds // 3)
    res = {"workers": 2, "data_size": 10, "max_chunk_size": 2, "max_lag": 1, "rounds": rounds,
           "transport": "tcp, one process per worker (cpu)"}
    # (tag, thComplete, assertMultiple, master transport, worker device, worker transport,
    #  workers, dataSize, maxChunkSize, maxLag)
    runs = [("demo_thresholds", 0.8, 0, "tcp", "cpu", None, 2, 10, 2, 1),
            ("exact_assert", 1.0, 2, "tcp", "cpu", None, 2, 10, 2, 1),
            # the reference's script config (scripts/testAllreduceMaster.sc:7-24):
            # 4 workers, 778 floats, 3-float chunks (65 per block), maxLag 3,
            # every round asserted x4 -- ~390 data messages per worker per round
            ("script_config_exact_assert", 1.0, 4, "tcp", "cpu", None, 4, 778, 3, 3)]
    if gpu:
        runs.append(("gpu_onesided_exact_assert", 1.0, 2, "onesided", "cuda", "onesided", 2, 10, 2, 1))
    for tag, thc, mult, mtransport, wdev, wtransport, nw, dsize, csize, lag in runs:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        with tempfile.TemporaryDirectory() as td:
            logs = [open(os.path.join(td, f"p{i}.log"), "w+") for i in range(nw + 1)]
            procs = [subprocess.Popen(base + ["master", "--port", str(port), "--workers", str(nw), "--data-size",
                                              str(dsize), "--max-chunk-size", str(csize), "--max-round", str(rounds),
                                              "--max-lag", str(lag),
                                              "--th-reduce", "1.0", "--th-complete", str(thc), "--transport",
                                              mtransport],
                                      stdout=logs[0], stderr=subprocess.STDOUT, cwd=os.path.dirname(__file__) or ".")]
            wd.watchdog_track_child(procs[0].pid)  # a watchdog exit of this rank takes the job down too
            t_end = time.time() + 20
            while time.time() < t_end:  # master listening?
                try:
                    socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                    break
                except OSError:
                    time.sleep(0.1)
            wextra = ["--transport", wtransport] if wtransport else []
            procs += [subprocess.Popen(base + ["worker", "--master", f"127.0.0.1:{port}", "--data-size", str(dsize),
                                               "--checkpoint", str(cp), "--assert-multiple", str(mult), "--device",
                                               wdev, *wextra], stdout=logs[i], stderr=subprocess.STDOUT,
                                       cwd=os.path.dirname(__file__) or ".") for i in range(1, nw + 1)]
            for p in procs[1:]:
                wd.watchdog_track_child(p.pid)
            rcs = []
            try:
                for p in procs:
                    rcs.append(p.wait(timeout=90))
            finally:
                for p in procs:
                    if p.poll() is None:
                        p.kill()
                        p.wait()
                    wd.watchdog_untrack_child(p.pid)
            entry = {"rcs": rcs, "rounds_per_s": [], "sink_MBps": [], "failures": [], "workers_on": wdev,
                     "data_plane": "one-sided lane (GPU windows)" if wtransport == "onesided" else "tcp"}
            if (nw, dsize, csize, lag) != (2, 10, 2, 1):
                entry.update({"workers": nw, "data_size": dsize, "max_chunk_size": csize, "max_lag": lag})
            for f in logs[1:]:
                f.seek(0)
                txt = f.read()
                el = [float(x) for x in re.findall(r"Mbytes in ([0-9.]+) seconds", txt)]
                mb = [float(x) for x in re.findall(r"at ([0-9.]+) MBytes/sec", txt)]
                fl = re.findall(r"failures=(\d+)", txt)
                entry["rounds_per_s"].append(round(cp / el[-1], 1) if el else None)
                entry["sink_MBps"].append(mb[-1] if mb else None)
                entry["failures"].append(int(fl[-1]) if fl else None)
            for f in logs:
                f.close()
            res[tag] = entry
    return res


def apply_lane_choice(ar, name) -> None:
    """Put a fresh ThresholdAllreduce on the lane the headline's lane selection
    chose (ThresholdAllreduce.LANES); None: leave auto."""
    if not name or ar.world_size < 2 or ar.transport != "stream":
        return
    if name.startswith("onesided"):
        try:
            ar.enable_onesided()  # collective; a failure on any rank raises on every rank
        except Exception as e:  # noqa: BLE001 - keep the job on the framework's p2p lane
            from akka_allreduce_amd.utils.phases import progress

            progress(f"rank {ar.rank}: onesided lane unavailable for this buffer ({type(e).__name__}: "
                     f"{str(e)[:120]}); the framework's p2p lane instead")
            ar.use_lane("p2p")
            ar.lane_fallback = f"onesided -> p2p ({type(e).__name__})"
            return
    if name.startswith("ipc") and not ar.state().get("link", {}).get("ipc"):
        try:
            ar.enable_ipc()  # collective; fails alike on every rank (e.g. a window too large for one mapping)
        except Exception as e:  # noqa: BLE001 - keep the job on the two-sided lanes
            from akka_allreduce_amd.utils.phases import progress

            progress(f"rank {ar.rank}: ipc lane unavailable for this buffer ({type(e).__name__}: {str(e)[:120]}); "
                     "the framework's p2p lane instead")
            # the framework's chunk-pipelined p2p schedule (gfx950 reduce), never
            # RCCL's own reduce-scatter + all-gather: that is the comparator
            ar.use_lane("p2p")
            ar.lane_fallback = f"{name} -> p2p ({type(e).__name__})"
            return
    ar.use_lane(name)


def _shareable(ar):
    """The headline engine if another exact-round engine can adopt its
    transport (stream transport, N > 1), else None."""
    if ar is None or getattr(ar, "transport", None) != "stream" or ar.world_size < 2 or ar.worker is None:
        return None
    return ar


def run_extras(world: int, dev, barrier, which=("cfg1", "cfg3", "cfg4", "cfg5"), rank: int = 0,
               cfg4_size_mb: float = 64.0, cfg4_delay_ms: float = 50.0, cfg4_rounds: int = 64,
               cfg4_transport: str = "onesided",
               lane: str | None = None, data_plane: str = "rccl", share=None) -> dict:
    """BASELINE config 3 (8-rank bf16, 1 GB buffer, link-sized chunks),
    config 4 (threshold 0.75/0.75 + straggler, N>1 only) and config 5 (2-layer
    MLP DP-SGD step/s) at this N, on synthetic data.  ``share``: the
    headline's ThresholdAllreduce; configs 3 and 5 ride on its transport
    (same device streams and communicator, its ipc windows where they fit)
    instead of adding streams -- hardware queues -- to the process."""
    import torch

    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.utils.phases import progress

    res: dict = {}
    keep = []  # communicators stay alive until exit (no per-rank teardown ordering)
    progress(f"rank {rank}: extras {','.join(which)}")
    if "cfg1" in which and rank == 0:
        try:
            res["cfg1_readme_demo_cluster"] = run_cfg1(gpu=dev.type == "cuda")
        except Exception as e:
            res["cfg1_error"] = f"{type(e).__name__}: {e}"[:200]
    if "cfg4" in which and world > 1:
        progress(f"rank {rank}: extra cfg4")
        try:
            if cfg4_transport == "onesided":
                res["cfg4_threshold_straggler"] = run_cfg4(world, rank, dev, barrier, cfg4_size_mb, cfg4_delay_ms,
                                                           cfg4_rounds)
            else:
                # the two-sided alternative: RCCL pair communicators, or the
                # mailbox p2p over mapped memory when the job runs without RCCL
                res["cfg4_threshold_straggler"] = run_cfg4_reactive(
                    world, rank, dev, barrier, cfg4_size_mb, cfg4_delay_ms, cfg4_rounds,
                    data_plane="rccl" if data_plane == "rccl" else "ipc_p2p")
        except Exception as e:
            res["cfg4_error"] = f"{type(e).__name__}: {e}"[:300]
    try:
        if "cfg3" not in which:
            raise _Skip()
        progress(f"rank {rank}: extra cfg3")
        nbytes = 1 << 30
        S = nbytes // 2
        ar = ThresholdAllreduce(S, max_chunk_size=(8 << 20) // 2, dtype=torch.bfloat16, device=dev,
                                data_plane=data_plane, share_transport_with=_shareable(share))
        keep.append(ar)
        apply_lane_choice(ar, lane)
        x = torch.randn(S, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(x)
        steps = 10
        dt = timed(lambda: ar(x, async_op=world > 1, out=out), steps, 3, world, barrier)
        link = ar.state().get("link", {}) if ar.world_size > 1 else {}
        ipc = link.get("ipc") or {}
        res["cfg3_bf16_1GiB_chunk8MiB"] = {"algbw_GBps": round(nbytes / (dt / steps) / 1e9, 3),
                                           "ms_per_step": round(dt / steps * 1e3, 4), "lane": link.get("lane"),
                                           "lane_fallback": getattr(ar, "lane_fallback", None),
                                           "lane_is_framework": link.get("lane") != "collective",
                                           "ipc_mode": {k: ipc.get(k) for k in ("mode", "fused", "lite", "max_wgs",
                                                                                "portions", "rounds",
                                                                                "shares_windows", "window_bytes")}
                                           if ipc else None}
        del x, out
    except _Skip:
        pass
    except Exception as e:
        res["cfg3_error"] = f"{type(e).__name__}: {e}"[:200]
    try:
        if "cfg5" not in which:
            raise _Skip()
        progress(f"rank {rank}: extra cfg5")
        from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
        from akka_allreduce_amd.parallel.dp import GradientBucket

        torch.manual_seed(0)  # identical init on every rank
        d_in, hidden, classes, batch = 4096, 8192, 1000, 256
        model = MLP(d_in, hidden, classes).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        # ranks on ONE card: a one-sided round waiting on its peers must leave
        # SIMDs free for the peers' GEMMs (OneSidedParams::cu_keep)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=(4 << 20) // 4, device=dev, data_plane=data_plane,
                                share_transport_with=_shareable(share),
                                onesided_options={"cu_keep": 6} if os.environ.get("AKKA_SHARE_GPU") == "1" else None)
        keep.append(ar)
        apply_lane_choice(ar, lane)
        gen = torch.Generator(device=dev).manual_seed(1000 + (ar.rank or 0))
        xb, yb = synthetic_batch(batch, d_in, classes, device=dev, generator=gen)
        steps = 20
        progress(f"rank {rank}: cfg5 eager fp32 (lane {(ar.state().get('link', {}) or {}).get('lane')})")
        dt = timed(lambda: dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False), steps, 5, world, barrier)
        res["cfg5_mlp_dp_sgd"] = {"steps_per_s": round(steps / dt, 3),
                                  "samples_per_s": round(steps * batch * world / dt, 1),
                                  "grad_bytes": bucket.numel * 4,
                                  "model": f"MLP {d_in}-{hidden}-{classes}, batch {batch}/rank",
                                  "compute_dtype": "fp32"}
        # same model/step with bf16 MFMA GEMMs (autocast); fp32 weights, grads,
        # allreduce and update
        progress(f"rank {rank}: cfg5 eager bf16")
        dt = timed(lambda: dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False,
                                       compute_dtype=torch.bfloat16), steps, 5, world, barrier)
        res["cfg5_mlp_dp_sgd_bf16"] = {"steps_per_s": round(steps / dt, 3),
                                       "samples_per_s": round(steps * batch * world / dt, 1),
                                       "compute_dtype": "bf16 autocast, fp32 master weights/grads"}
        # same step with forward + backward replayed from a HIP graph (the
        # allreduce and the fused update stay eager: GraphedDPStep)
        from akka_allreduce_amd.models.mlp import GraphedDPStep

        progress(f"rank {rank}: cfg5 graphed forward+backward")
        gstep = GraphedDPStep(model, bucket, xb, yb, compute_dtype=torch.bfloat16)
        gx, gy = gstep.static_inputs()  # the synthetic batch lives in the graph's buffers
        dt = timed(lambda: gstep(gx, gy, 0.05, ar), steps, 5, world, barrier)
        res["cfg5_mlp_dp_sgd_bf16_graph"] = {"steps_per_s": round(steps / dt, 3),
                                             "samples_per_s": round(steps * batch * world / dt, 1),
                                             "compute_dtype": "bf16 autocast, fp32 master weights/grads; "
                                                              "forward+backward as one HIP graph replay"}
        # N > 1 on a window lane (ipc* / onesided): the WHOLE step -- forward,
        # backward, the allreduce and the fused average + SGD update -- as one
        # replay (device-resident round ids, ThresholdAllreduce.capturable())
        chosen = (ar.state().get("link", {}) or {}).get("lane") if world > 1 else None
        if world > 1 and chosen is not None and (str(chosen).startswith("ipc") or str(chosen).startswith("onesided")):
            _sync()
            barrier()
            progress(f"rank {rank}: cfg5 whole step graphed ({chosen})")
            cap = ar.capturable()
            try:
                wstep = GraphedDPStep(model, bucket, xb, yb, compute_dtype=torch.bfloat16, allreduce=cap, lr=0.05)
                wx, wy = wstep.static_inputs()
                dt = timed(lambda: wstep(wx, wy, 0.05, None), steps, 5, world, barrier)
                res["cfg5_mlp_dp_sgd_bf16_whole_graph"] = {
                    "steps_per_s": round(steps / dt, 3), "samples_per_s": round(steps * batch * world / dt, 1),
                    "lane": lane or chosen, "compute_dtype": "bf16 autocast, fp32 master weights/grads; forward, backward, "
                                                     "allreduce and update as one HIP graph replay"}
            finally:
                _sync()
                barrier()
                cap.close()
    except _Skip:
        pass
    except Exception as e:
        res["cfg5_error"] = f"{type(e).__name__}: {e}"[:200]
    run_extras.keep = keep  # type: ignore[attr-defined]
    return res


def _identity(ar, dev) -> dict:
    """What this rank runs on, as the transport itself reports it (RCCL:
    ncclCommCount / ncclCommUserRank / ncclCommCuDevice)."""
    import torch

    d = {"rank": ar.rank}
    if dev.type == "cuda":
        props = torch.cuda.get_device_properties(dev)
        d["hip_device"] = dev.index
        d["pci_bus_id"] = getattr(props, "pci_bus_id", None)
        d["gpu"] = props.name
    p2p = ar.worker._core.p2p_info()
    if p2p is not None:
        d["p2p"] = p2p
    return d


def main() -> int:
    args = parse()
    if args.transport == "reactive":
        # one stream per peer: must not share hardware queues (read at HIP init)
        os.environ["GPU_MAX_HW_QUEUES"] = "32"
    elif int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # comm + compute + caller (+ RCCL's own) streams each on their own
        # hardware queue, so chunk reduces never serialise behind transfers;
        # config 4 (reactive transport, run first among the extras) adds one
        # stream per peer + comm + compute on top of the headline worker's two,
        # torch's default stream and the comparator's RCCL stream: N + 8 keeps
        # every stream on its own hardware queue (a stream parked on the
        # straggler must not hold up a reduce that shares its queue)
        need = min(32, max(8, int(os.environ["WORLD_SIZE"]) + 8))
        # ranks sharing one card (rehearsal) split its hardware queues: keep the caller's setting
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < need and os.environ.get("AKKA_SHARE_GPU") != "1":
            os.environ["GPU_MAX_HW_QUEUES"] = str(need)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
        print(f"bench.py: --gpus {args.gpus} needs torch.distributed.run (WORLD_SIZE unset)", file=sys.stderr)
        return 2
    from akka_allreduce_amd.utils.faults import env_phase_stall
    from akka_allreduce_amd.utils.phases import PhaseGuard, enable_rccl_debug_log

    # RCCL warnings go to a per-rank file whose tail a failure line carries
    debug_path = enable_rccl_debug_log(rank) if (world > 1 and args.device == "cuda") else ""
    import torch
    import torch.distributed as dist

    dtype = torch.float32 if args.dtype == "float32" else torch.bfloat16
    esize = 4 if dtype == torch.float32 else 2
    nbytes = int(args.size_mb * (1 << 20))
    S = nbytes // esize
    C = max(1, int(args.chunk_mb * (1 << 20)) // esize)
    base = {
        "metric": BASELINE_METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "higher_is_better": True,
        # a fixed 256 MiB buffer whatever N is: total work is fixed (strong scaling)
        "scaling": "strong", "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic random tensors (torch.randn), exact thresholds"
        + ("; CPU gloo rehearsal, not the metric" if args.device == "cpu" else ""),
        "config": {
            "model": f"threshold-allreduce {args.size_mb:g}MiB {args.dtype}",
            "global_batch": world, "seq_len": S, "parallelism": f"dp{world}", "buffer_bytes": nbytes,
            "chunk_bytes": C * esize, "max_lag": args.max_lag, "broadcast_lag": args.bcast_lag,
            "thresholds": [1.0, args.th_reduce, args.th_complete],
        },
    }
    # stdout carries exactly ONE line, this rank-0 JSON line: everything else
    # that writes to fd 1 (gloo's connection banners, RCCL's version banner,
    # stray prints of any rank) goes to stderr from here on.  The real stdout
    # stays reachable through a private descriptor, for the result line and
    # for the native watchdog's failure line.
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    json_out = os.fdopen(out_fd, "w", buffering=1)
    from akka_allreduce_amd._native_loader import load as _load_native

    _load_native().watchdog_set_out_fd(out_fd)
    guard = PhaseGuard(base, rank, world, debug_path, stream=json_out)
    dl = args.phase_deadline_s

    def init():
        env_phase_stall(rank, "init")
        if args.device == "cpu":
            dev = torch.device("cpu")
        else:
            if not torch.cuda.is_available():
                raise RuntimeError("no GPU visible")
            loc = local
            if os.environ.get("AKKA_SHARE_GPU") == "1":
                # rehearsal only: several ranks on one card (1-GPU box)
                loc %= max(1, torch.cuda.device_count())
            torch.cuda.set_device(loc)
            dev = torch.device("cuda", loc)
        if world > 1:
            from datetime import timedelta

            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=args.pg_timeout_s))
        return dev

    dev = guard.run("init", dl, init, agree=False)
    if args.watchdog_s > 0:
        # outer bound on the whole run (stacks + exit) on top of the phase deadlines
        import faulthandler

        faulthandler.dump_traceback_later(args.watchdog_s, exit=True)

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    # The extras' exact-round engines ride on the headline engine's transport
    # (run_extras(share=...)); its ipc windows are sized for config 3's 1 GiB
    # so that engine reuses them too: a second window set mapped by every
    # process slowed whole rounds by 4-20x when ranks share one card
    # (profiles/r03/README.md), and costs mappings on a node.
    will_cfg3 = (world > 1 and args.transport == "stream" and args.device == "cuda"
                 and (args.extras == "on" or (args.extras == "auto" and args.size_mb == 256.0
                                              and args.dtype == "float32"))
                 and (not args.extras_only or "cfg3" in args.extras_only.split(",")))
    ipc_cap = max(S, (1 << 30) // esize) if will_cfg3 else 0

    # the headline's one-sided lane (an exact tune candidate) returns its
    # window row when called without ``out``: the peers' reduced parts land
    # in place, no copy into a caller buffer (the line's config.output says
    # which output the timed rounds used)
    os_opts = {"window_output": True} if args.lane_output == "on" else None

    def rccl_init():
        env_phase_stall(rank, "rccl_init")
        return ThresholdAllreduce(S, max_chunk_size=C, dtype=dtype, th_reduce=args.th_reduce,
                                  th_complete=args.th_complete, max_lag=args.max_lag, broadcast_lag=args.bcast_lag,
                                  device=dev, transport=args.transport, lane=args.lane,
                                  data_plane=args.data_plane, ipc_capacity=ipc_cap, onesided_options=os_opts)

    # RCCL failing on EVERY rank (agreed) does not cost the headline: the job
    # is rebuilt in this same process on the ipc data plane (one-sided xGMI,
    # no RCCL communicator at all) and the line says so.  A failure on some
    # ranks only, or a hang, still ends the job with the failure line.
    ar, init_errors = guard.try_run("rccl_init", dl, rccl_init)
    rccl_fallback = None
    if init_errors:
        if (len(init_errors) == world and world > 1 and args.data_plane == "rccl" and dev.type == "cuda"
                and args.transport == "stream"):
            rccl_fallback = {"rccl_init_errors": {str(k): v[:200] for k, v in init_errors.items()},
                             "data_plane": "ipc"}
            args.data_plane = "ipc"
            ar = guard.run("ipc_init", dl, lambda: ThresholdAllreduce(
                S, max_chunk_size=C, dtype=dtype, max_lag=args.max_lag, broadcast_lag=args.bcast_lag, device=dev,
                data_plane="ipc", ipc_capacity=ipc_cap, onesided_options=os_opts))
        else:
            guard.fail("rccl_init", "error", init_errors)

    def identity():
        me = _identity(ar, dev)
        if world == 1:
            return [me]
        allv = [None] * world
        dist.all_gather_object(allv, me)
        for d in allv:
            p2p = d.get("p2p") or {}
            if p2p.get("kind", "").startswith("rccl") and (p2p.get("nranks") != world or p2p.get("rank") != d["rank"]):
                raise RuntimeError(f"rank {d['rank']}: RCCL reports nranks={p2p.get('nranks')} rank={p2p.get('rank')}")
        return allv

    ranks = guard.run("identity", dl, identity)
    p2p0 = ranks[0].get("p2p") or {}
    rccl_kind = str(p2p0.get("kind", "")).startswith("rccl")

    def barrier():
        if world > 1:
            dist.barrier()

    def exact_round(tag: str, salt: int = 0) -> bool:
        # every rank contributes (rank+1)(salt+1) -> sum = (salt+1) N(N+1)/2 exactly, count N
        y = torch.full((S,), float((rank + 1) * (salt + 1)), device=dev, dtype=dtype)
        o = ar(y)
        want = float((salt + 1) * world * (world + 1) // 2)
        ok = bool(torch.all(o.data == want).item()) and bool(torch.all(o.count == world).item())
        if world > 1:
            f = torch.tensor([1 if ok else 0])
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = bool(f.item())
        return ok

    def preflight():
        # one exact full-size round before anything is timed: a hang or a wrong
        # sum shows up here, under its own deadline, with its own failure line
        env_phase_stall(rank, "preflight")  # fault injection (AKKA_FAULT_STALL_*): stall or raise here
        if not exact_round("preflight"):
            raise RuntimeError("preflight round is not exact (sum or counts differ on some rank)")
        return True

    # A preflight that fails on EVERY rank (an error or a wrong sum, agreed) on
    # the two-sided default lane does not cost the headline either: the job
    # moves to the one-sided ipc lane (no RCCL kernel involved) and checks it
    # with its own exact round; lane selection then only tries ipc lanes.  A
    # failure on some ranks only, or a hang, still ends the job.
    preflight_fallback = None
    ipc_only = False
    failed_engines: list = []
    if world > 1 or args.preflight == "on":
        can_fall_back = (world > 1 and dev.type == "cuda" and ar.transport == "stream"
                         and args.data_plane != "ipc" and args.ipc == "on")
        if can_fall_back:
            _, pf_errors = guard.try_run("preflight", args.preflight_deadline_s, preflight)
            if pf_errors and len(pf_errors) == world:
                preflight_fallback = {"errors": {str(k): v[:200] for k, v in pf_errors.items()},
                                      "lane": "ipc_fused_lite"}

                def preflight_ipc():
                    nonlocal ar
                    # a FRESH engine on the ipc data plane (no RCCL communicator):
                    # the failed engine's comm stream may still hold failed or
                    # queued RCCL work and its round state is suspect, so it is
                    # kept alive (never torn down mid-failure) but not reused
                    failed_engines.append(ar)
                    ar = ThresholdAllreduce(S, max_chunk_size=C, dtype=dtype, max_lag=args.max_lag,
                                            broadcast_lag=args.bcast_lag, device=dev, data_plane="ipc",
                                            ipc_capacity=ipc_cap, onesided_options=os_opts)
                    ar.use_lane("ipc_fused_lite")
                    if not exact_round("preflight_ipc"):
                        raise RuntimeError("ipc preflight round is not exact")
                    return True

                guard.run("preflight_ipc", args.preflight_deadline_s, preflight_ipc)
                ipc_only = True
                args.data_plane = "ipc"
            elif pf_errors:
                guard.fail("preflight", "error", pf_errors)
        else:
            guard.run("preflight", args.preflight_deadline_s, preflight)

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    x = torch.randn(S, device=dev, dtype=torch.float32, generator=g).to(dtype)

    # Rounds are issued back to back (async_op, like nccl-tests / torch's
    # async_op=True): every round's output is waited for on the current stream
    # before the closing synchronize, so all K rounds complete inside the timing.
    # The output goes into one preallocated buffer reused every round (like
    # nccl-tests' recvbuff): all rounds run in order on the engine's streams, so
    # waiting for the last round's event covers every round.
    out_buf = None if args.fresh_out else torch.empty(S, device=dev, dtype=dtype)
    args.async_op = (world > 1) if args.async_op == "auto" else (args.async_op == "on")
    if ar.transport == "reactive":
        args.async_op = False  # reactive rounds return once complete (progress is host-polled)

    # Lane selection (untimed, before the warmup): every exact-round lane of
    # the stream transport computes the same exact sum -- RCCL reduce-scatter +
    # all-gather, the chunk-pipelined direct p2p schedule with our reduce
    # kernel (16 MiB or whole-block units), or the one-sided ipc kernels over
    # mapped peer windows (four variants).  Which is fastest depends on N, the
    # xGMI topology and the buffer, so ThresholdAllreduce.tune checks each for
    # exactness and times it on this job; every rank agrees on the result.
    chosen_lane = args.lane if args.lane != "auto" else None

    def lane_select():
        env_phase_stall(rank, "lane_select")
        # (ipc_only: the two-sided lane failed its preflight; the engine on the
        # ipc data plane has no p2p lane, so the window lanes alone compete)
        return ar.tune(try_ipc=args.ipc == "on" or ipc_only)

    lane_sel = None
    if world > 1 and ar.transport == "stream" and args.lane == "auto" and args.lane_select == "on":
        lane_sel = guard.run("lane_select", dl, lane_select)
        chosen_lane = lane_sel["chosen"]

    if out_buf is not None and ar.world_size > 1 and ar.prefers_lane_output():
        out_buf = None  # the chosen lane's own output (window row, valid until the next round)
        lane_output = True
    else:
        lane_output = False

    def warmup():
        env_phase_stall(rank, "warmup")
        out = None
        for _ in range(args.warmup):
            out = ar(x, async_op=args.async_op, out=out_buf)
        if out is not None:
            out.wait()
        _sync()
        barrier()
        _sync()

    guard.run("warmup", dl, warmup)

    link0 = dict(ar.state().get("link", {}))  # counters before the timed rounds

    def timed_region():
        env_phase_stall(rank, "timed")
        host_s = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            th = time.perf_counter()
            out = ar(x, async_op=args.async_op, out=out_buf)
            host_s += time.perf_counter() - th
        out.wait()
        _sync()
        barrier()
        _sync()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt, host_s], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt, host_s = float(t[0].item()), float(t[1].item())
        return dt, host_s

    dt, host_s = guard.run("timed", max(dl, args.steps * 2.0), timed_region)
    ms = dt / args.steps * 1e3
    algbw = nbytes / (dt / args.steps) / 1e9
    busbw = algbw * (2 * (world - 1) / world) if world > 1 else None

    # Exactness after the timed rounds (untimed).
    ok = None
    if not args.no_check:
        ok = guard.run("check", dl, lambda: exact_round("check"))

    # Comparator (outside the timed region): RCCL's own all_reduce on the same
    # buffer, same N and step count, through a separate nccl (= RCCL) group.
    compare = (world > 1) if args.compare_rccl == "auto" else (args.compare_rccl == "on")
    if ipc_only:
        compare = False  # RCCL failed the preflight: no RCCL comparator after the headline

    def comparator():
        if not (compare and world > 1):
            return None, None
        try:
            grp = dist.new_group(backend="nccl" if dev.type == "cuda" else "gloo")
            z = x.clone()
            for _ in range(args.warmup):
                dist.all_reduce(z, group=grp)
            _sync()
            barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                dist.all_reduce(z, group=grp)
            _sync()
            barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            del z
            return nbytes / (float(t.item()) / args.steps) / 1e9, None
        except Exception as e:  # the comparator must never cost the headline line
            return None, f"{type(e).__name__}: {e}"[:200]

    rccl, rccl_err = guard.run("compare", dl, comparator)

    # The other exact-round lane on the same buffer (untimed for the headline):
    # at N>1 the driver's run then records both the whole-round collective lane
    # and the chunk-pipelined p2p schedule.
    def other_lane():
        st0 = ar.state().get("link", {})
        # lane of the timed rounds: collective rounds vs exact p2p-step rounds since link0
        coll = st0.get("collective_rounds", 0) - link0.get("collective_rounds", 0)
        steps_p2p = st0.get("exact_step_rounds", 0) - link0.get("exact_step_rounds", 0)
        used = chosen_lane or ("ipc" if args.data_plane == "ipc" else "collective" if coll > steps_p2p else "p2p")
        if world == 1:
            return "local", None
        if args.data_plane == "ipc" or ipc_only:
            return used, None
        if ar.transport != "stream":
            return used, None
        other = "p2p" if used == "collective" else "collective"
        try:
            ar.use_lane(other)
            for _ in range(2):
                o = ar(x, async_op=args.async_op, out=out_buf)
            o.wait()
            _sync()
            barrier()
            k = max(3, args.steps // 2)
            t0 = time.perf_counter()
            for _ in range(k):
                o = ar(x, async_op=args.async_op, out=out_buf)
            o.wait()
            _sync()
            barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return used, {"lane": other, "algbw_GBps": round(nbytes / (float(t.item()) / k) / 1e9, 3),
                          "steps": k}
        finally:
            if chosen_lane or args.lane != "auto":
                ar.use_lane(chosen_lane or args.lane)
            else:
                ar.set_lane("auto")

    st = ar.state()  # headline rounds only (before the other lane runs)
    lane_used, lane_other = guard.run("other_lane", dl, other_lane)

    link = st.get("link", {})
    # per-round link counters of the timed rounds only (plus the check round)
    rounds_done = max(1, link.get("rounds", 0) - link0.get("rounds", 0))
    line = dict(base)
    line.update({
        "value": round(algbw, 3),
        "ms_per_step": round(ms, 4),
        "busbw_GBps": round(busbw, 3) if busbw is not None else None,
        "exact": ok,
        "preflight": ("passed" if "preflight" in guard.history else
                      "passed on the ipc lane" if "preflight_ipc" in guard.history else "skipped"),
        "groups_per_round": round((link.get("groups", 0) - link0.get("groups", 0)) / rounds_done, 3),
        "host_us_per_round": round(host_s / args.steps * 1e6, 2),
        "p2p_kind": p2p0.get("kind"),
        "p2p_nranks": p2p0.get("nranks"),
        "rccl_nranks": p2p0.get("nranks") if rccl_kind else None,
        "rccl_version": _rccl_version() if rccl_kind else None,
        "rank_devices": ranks,
        "lane": lane_used,
        # the headline's lane is one of the framework's (p2p schedule with the
        # gfx950 reduce, or the one-sided ipc kernels) unless --lane collective
        # forced RCCL's own reduce-scatter + all-gather
        "lane_is_framework": lane_used != "collective",
        "other_lane": lane_other,
        "lane_select": lane_sel,
        "rccl_allreduce_algbw_GBps": round(rccl, 3) if rccl else None,
    })
    line["config"] = dict(base["config"])
    line["config"].update({
        "transport": ("xgmi-ipc" if str(lane_used).startswith("ipc") else
                      "xgmi-onesided" if str(lane_used).startswith("onesided") else
                      "xgmi-mailbox-p2p" if args.data_plane == "ipc_p2p" else
                      "rccl-pair-reactive" if ar.transport == "reactive" else "rccl-p2p-xgmi")
        if world > 1 and dev.type == "cuda" else ("gloo-p2p" if world > 1 else "local"),
        # N=1 moves nothing between ranks: no data plane runs
        "data_plane": args.data_plane if world > 1 else "none (local reduce pass)",
        "async_op": args.async_op,
        "output": ("the lane's window row, valid until the next round (no copy into a caller buffer)"
                   if lane_output else "fresh tensor per round" if args.fresh_out else "preallocated, reused"),
    })
    if rccl_err:
        line["rccl_compare_error"] = rccl_err
    if rccl_fallback:
        line["rccl_fallback"] = rccl_fallback
    if preflight_fallback:
        line["preflight_fallback"] = preflight_fallback
    if os.environ.get("AKKA_SHARE_GPU") == "1" and world > 1:
        line["data"] += "; N ranks sharing ONE GPU (rehearsal of the N-rank flow, not the metric)"
    if world == 1:
        line["note"] = ("N=1 has no peer: the round is one local reduce pass (input -> output), HBM-bound; "
                        "N>1 is xGMI-bound, compare it with rccl_allreduce_algbw_GBps")
        line["host_us_note"] = ("N=1: host time of one launch on the caller's stream; at N>1 it is the engine's "
                                "per-round scheduling (transfers + reduces), not comparable")
    else:
        # direct scatter/broadcast moves S/N per link per phase: algbw <= N*L/2
        line["xgmi_bound_algbw_GBps"] = round(world * XGMI_LINK_GBPS / 2, 1)

    # Per-link probe (N>1, untimed, after the headline): every ordered pair's
    # remote-write (push) and remote-read (pull) bandwidth through mapped
    # memory, and every rank to all peers at once.  It validates the ~153 GB/s
    # per xGMI link behind xgmi_bound_algbw_GBps.  Bounded like the extras: a
    # hang prints the headline line with link_probe_error instead.
    if world > 1 and args.link_probe == "on":
        late = dict(line)
        late["link_probe_error"] = f"link probe not done after {args.link_probe_deadline_s:g} s; skipped"
        guard.arm(args.link_probe_deadline_s, late, exit_code=0 if ok in (None, True) else 1)
        progress_msg = f"rank {rank}: link probe"
        from akka_allreduce_amd.utils.phases import progress

        progress(progress_msg)
        try:
            from akka_allreduce_amd.utils.link_probe import probe_links

            probe = probe_links(rank, world, dev, mib=args.link_probe_mib, iters=3)
            if rank == 0:
                if dev.type != "cuda":
                    probe["note"] = "CPU shared memory (gloo rehearsal): not a link measurement"
                elif os.environ.get("AKKA_SHARE_GPU") == "1":
                    probe["note"] = "ranks share ONE GPU: copies inside one card's HBM, not xGMI"
                else:
                    probe["note"] = "one rank per GPU: each pair is an xGMI link"
                line["link_probe"] = probe
        except Exception as e:  # noqa: BLE001 - the probe must never cost the headline
            line["link_probe_error"] = f"{type(e).__name__}: {e}"[:200]
        guard.disarm()

    # The other BASELINE configs at the same N, measured after the headline
    # (each guarded so it cannot cost the line).  The native watchdog bounds
    # them: if they have not finished by the deadline, every rank exits and
    # rank 0 writes the headline line with "extras_error" instead.
    run_extra = args.extras == "on" or (args.extras == "auto" and args.size_mb == 256.0 and args.dtype == "float32"
                                        and args.transport == "stream" and dev.type == "cuda")
    if run_extra:
        late = dict(line)
        late["extras_error"] = f"extras not done after {args.extras_deadline_s:g} s; skipped"
        guard.arm(args.extras_deadline_s, late, exit_code=0 if ok in (None, True) else 1)
        which = tuple(args.extras_only.split(",")) if args.extras_only else ("cfg1", "cfg3", "cfg4", "cfg5")
        line["extra_configs"] = run_extras(world, dev, barrier, which, rank, args.cfg4_size_mb,
                                           args.cfg4_delay_ms, args.cfg4_rounds, cfg4_transport=args.cfg4_transport,
                                           lane=chosen_lane,
                                           data_plane=args.data_plane, share=ar)
        if chosen_lane and world > 1:
            line["extra_configs"]["lane"] = chosen_lane
        guard.disarm()

    if world > 1:
        # the job's own correctness checks in one place (on a node: the
        # cross-device hand-offs of the window lanes)
        sel = line.get("lane_select") or {}
        v4 = ((line.get("extra_configs") or {}).get("cfg4_threshold_straggler") or {}).get("validation") or {}
        line["checks"] = {
            "headline_exact": line.get("exact"),
            "preflight": line.get("preflight"),
            "lane_candidates_exact": sorted(k for k, v in sel.items() if isinstance(v, dict) and v.get("exact")),
            "lane_candidates_rejected": sorted(k for k, v in sel.items() if isinstance(v, dict) and not v.get("exact")),
            "cfg4_contributor_sets_consistent": v4.get("contributor_sets_consistent"),
            "cfg4_chunks_checked": v4.get("chunks_checked"),
        }

    if rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    if world > 1 and dist.is_initialized():
        guard.run("teardown", dl, lambda: (dist.barrier(), dist.destroy_process_group()), agree=False)
    return 0 if ok in (None, True) else 1


def _rccl_version():
    from akka_allreduce_amd._native_loader import load

    return load().rccl_version()


if __name__ == "__main__":
    sys.exit(main())
