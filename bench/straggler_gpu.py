#!/usr/bin/env python3
"""Straggler tolerance on one MI355X: N loopback ranks (threads, each with its
own HIP streams / data plane / link), rank N-1 sleeps `--delay-ms` before
every round.  Reports how long the fast ranks take for R rounds with

  * the scheduled transport (StreamLink: symmetric all-peer groups -- every
    rank proceeds at the pace of the slowest), and
  * the reactive transport (ReactiveLink: per-peer streams, event-polled
    arrivals -- thresholds < 1 let the fast ranks finish without the straggler,
    bounded by the send-slot pool).

Both at thReduce = thComplete = --th.  One JSON line per mode.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

os.environ["GPU_MAX_HW_QUEUES"] = "32"  # per-peer streams must not share hardware queues
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd.messages import InitWorkers  # noqa: E402
from akka_allreduce_amd.parallel.collective import _RemoteRank  # noqa: E402
from akka_allreduce_amd.worker import AllreduceWorker  # noqa: E402


def run(mode: str, n: int, S: int, C: int, th: float, rounds: int, delay: float, max_lag: int):
    from akka_allreduce_amd._native_loader import load

    nat = load()
    if mode == "stream":
        hub = nat.LoopbackHub(n)
        spec = lambda r: ("loopback", hub, r)  # noqa: E731
    else:
        hub = nat.PairLoopbackHub(n)
        spec = lambda r: ("loopback_pair", hub, r)  # noqa: E731
    dev = torch.device("cuda", 0)
    ws = [AllreduceWorker(None, None, device=dev, transport=mode, transport_spec=spec(r), strict=True,
                          name=f"{mode}{r}") for r in range(n)]
    for r, w in enumerate(ws):
        w.reactive_timeout = 120.0
        peers = {i: (w if i == r else _RemoteRank(i)) for i in range(n)}
        w.tell(InitWorkers(peers, n, None, r, th, th, max_lag, S, C))
    xs = [torch.full((S,), float(1 << r), device=dev) for r in range(n)]
    # warm-up round (all ranks, no delay)
    finish = [0.0] * n
    counts = [[] for _ in range(n)]
    stamps = [[] for _ in range(n)]
    errs = []

    def body(r, nrounds, sleep, t0):
        try:
            for _ in range(nrounds):
                if sleep:
                    time.sleep(sleep)
                o = ws[r].allreduce(xs[r])
                counts[r].append(o.count[0].item() if r == 0 else 0)
                stamps[r].append(round((time.perf_counter() - t0) * 1e3, 2))
            torch.cuda.current_stream().synchronize()
            finish[r] = time.perf_counter() - t0
        except BaseException as e:  # pragma: no cover
            errs.append(e)

    def phase(nrounds, sleeps):
        t0 = time.perf_counter()
        ts = [threading.Thread(target=body, args=(r, nrounds, sleeps[r], t0)) for r in range(n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]

    phase(2, [0.0] * n)
    for c in counts + stamps:
        c.clear()
    phase(rounds, [0.0] * (n - 1) + [delay])
    res = {
        "mode": mode, "n": n, "bytes": S * 4, "threshold": th, "rounds": rounds, "straggler_delay_ms": delay * 1e3,
        "fast_ranks_s": round(max(finish[: n - 1]), 4), "straggler_s": round(finish[n - 1], 4),
        "fast_ms_per_round": round(max(finish[: n - 1]) / rounds * 1e3, 3),
        "rank0_first_chunk_counts": counts[0],
        "round_done_ms": {r: stamps[r] for r in (0, n - 1)},
    }
    if mode == "reactive":
        for w in ws:  # drain and free deterministically (hipFree syncs the device)
            t0 = time.monotonic()
            while w._core.in_flight() and time.monotonic() - t0 < 30:
                for v in ws:
                    v.poll()
        res["link"] = ws[0].state()["link"]
    for w in ws:
        w.close()
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=3)
    p.add_argument("--size-mb", type=float, default=16)
    p.add_argument("--chunk-mb", type=float, default=1)
    p.add_argument("--th", type=float, default=0.67)
    p.add_argument("--rounds", type=int, default=10)
    p.add_argument("--delay-ms", type=float, default=50)
    p.add_argument("--max-lag", type=int, default=2)
    p.add_argument("--modes", default="stream,reactive")
    a = p.parse_args()
    S = int(a.size_mb * (1 << 20)) // 4
    C = int(a.chunk_mb * (1 << 20)) // 4
    modes = a.modes.split(",")
    if len(modes) > 1:
        # one fresh process per mode: no leftover streams/queues from the other
        import subprocess

        rc = 0
        for mode in modes:
            argv = [sys.executable, os.path.abspath(__file__)] + [x for x in sys.argv[1:]]
            if "--modes" in argv:
                i = argv.index("--modes")
                del argv[i:i + 2]
            rc |= subprocess.run(argv + ["--modes", mode]).returncode
        sys.exit(rc)
    print(json.dumps(run(modes[0], a.n, S, C, a.th, a.rounds, a.delay_ms / 1e3, a.max_lag)), flush=True)


if __name__ == "__main__":
    main()
