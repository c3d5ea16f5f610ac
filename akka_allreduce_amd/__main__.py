"""Command line: ``python -m akka_allreduce_amd {master,worker,demo,info}``.

Reference CLIs (README.md:3-7, M:95-112, W:309-315):
  master [port=2551] [totalWorkers=2] [dataSize=totalWorkers*5] [maxChunkSize=2]
  worker [port=2553] [dataSize=10]
The same positional forms work here; every other parameter (thresholds,
maxLag, maxRound -- hardcoded in the reference, README.md:5) is a flag or
comes from the config file (conf/application.yaml, AKKA_* env vars).
"""
from __future__ import annotations

import argparse
import logging
import subprocess
import sys
import time

from .config import DataConfig, ThresholdConfig, WorkerConfig, load_config


def _master(a: argparse.Namespace) -> int:
    from .parallel.cluster import start_master

    cfg = load_config(a.config)
    port = a.port if a.port is not None else (a.pos[0] if len(a.pos) > 0 else cfg.cluster.port)
    total = a.workers if a.workers is not None else (a.pos[1] if len(a.pos) > 1 else cfg.workers.totalSize)
    size = a.data_size if a.data_size is not None else (a.pos[2] if len(a.pos) > 2 else total * 5)
    chunk = a.max_chunk_size if a.max_chunk_size is not None else (a.pos[3] if len(a.pos) > 3 else cfg.data.maxChunkSize)
    th = ThresholdConfig(
        a.th_allreduce if a.th_allreduce is not None else cfg.thresholds.thAllreduce,
        a.th_reduce if a.th_reduce is not None else cfg.thresholds.thReduce,
        a.th_complete if a.th_complete is not None else cfg.thresholds.thComplete,
    )
    th.validate()
    data = DataConfig(int(size), int(chunk), a.max_round if a.max_round is not None else cfg.data.maxRound)
    wc = WorkerConfig(int(total), a.max_lag if a.max_lag is not None else cfg.workers.maxLag)
    m = start_master(th, data, wc, host=a.host or cfg.cluster.host, port=int(port),
                     heartbeat_interval_s=cfg.cluster.heartbeat_interval_s,
                     unreachable_after_s=cfg.cluster.unreachable_after_s, transport=a.transport or cfg.engine.transport,
                     min_workers=a.min_workers)
    print(f"-------\n Port = {m.node.port} \n Number of Workers = {wc.totalSize} \n Message Size = {data.dataSize} "
          f"\n Max Chunk Size = {data.maxChunkSize}", flush=True)
    try:
        while not m.wait(0.5):
            pass
        time.sleep(0.5)  # let Shutdown reach the workers
    except KeyboardInterrupt:
        pass
    m.stop()
    return 0


def _worker(a: argparse.Namespace) -> int:
    import os

    if a.transport == "reactive" and os.environ.get("AKKA_SHARE_GPU") != "1":
        # one stream per peer: they must not share hardware queues (read at HIP
        # init); workers sharing one card split its queues: keep their setting
        os.environ["GPU_MAX_HW_QUEUES"] = "32"
    import torch

    from .parallel.cluster import start_worker

    cfg = load_config(a.config)
    port = a.port if a.port is not None else (a.pos[0] if len(a.pos) > 0 else 0)
    size = a.data_size if a.data_size is not None else (a.pos[1] if len(a.pos) > 1 else 10)
    master = a.master or f"{cfg.cluster.host}:{cfg.cluster.port}"
    dtype = torch.bfloat16 if a.dtype in ("bf16", "bfloat16") else torch.float32
    device = a.device or cfg.engine.device
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    w = start_worker(master, int(size), checkpoint=a.checkpoint if a.checkpoint is not None else cfg.checkpoint,
                     assert_multiple=a.assert_multiple, port=int(port), device=device, dtype=dtype,
                     transport=a.transport, host=a.host or "127.0.0.1",
                     metrics_interval_s=cfg.cluster.metrics_interval_s)
    try:
        while not w.wait(0.5):
            pass
    except KeyboardInterrupt:
        w.stop()
    sink = w.worker.dataSink
    failures = getattr(sink, "failures", 0)
    print(f"worker {w.worker.id}: rounds={getattr(sink, 'rounds', '?')} failures={failures}", flush=True)
    return 1 if failures else 0


def _demo(a: argparse.Namespace) -> int:
    """Master + N worker processes on localhost (README demo / scripts/*.sc)."""
    base = [sys.executable, "-m", "akka_allreduce_amd"]
    mport = a.port
    master = subprocess.Popen(base + ["master", "--port", str(mport), "--workers", str(a.workers), "--data-size",
                                      str(a.data_size), "--max-chunk-size", str(a.max_chunk_size), "--max-round",
                                      str(a.max_round), "--max-lag", str(a.max_lag), "--th-complete",
                                      str(a.th_complete), "--th-reduce", str(a.th_reduce), "--transport", "tcp"])
    time.sleep(1.0)
    workers = [subprocess.Popen(base + ["worker", "--master", f"127.0.0.1:{mport}", "--data-size", str(a.data_size),
                                        "--checkpoint", str(a.checkpoint), "--assert-multiple",
                                        str(a.assert_multiple), "--device", "cpu"]) for _ in range(a.workers)]
    rc = 0
    try:
        for p in workers:
            rc |= p.wait(timeout=a.timeout)
        rc |= master.wait(timeout=a.timeout)
    finally:  # a timeout or ^C must not leave the master or a worker behind
        for p in [master, *workers]:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def _info(_a: argparse.Namespace) -> int:
    import torch

    from . import _native_loader

    n = _native_loader.load()
    print(f"native core: arch={n.build_arch} rccl={n.rccl_version()}")
    print(f"torch {torch.__version__} hip={torch.version.hip} gpus={torch.cuda.device_count()}")
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="akka_allreduce_amd")
    p.add_argument("--log-level", default="INFO")
    sub = p.add_subparsers(dest="cmd", required=True)

    m = sub.add_parser("master", help="run the AllreduceMaster")
    m.add_argument("pos", nargs="*", type=int, help="[port] [totalWorkers] [dataSize] [maxChunkSize]")
    m.add_argument("--config")
    m.add_argument("--host")
    m.add_argument("--port", type=int)
    m.add_argument("--workers", type=int)
    m.add_argument("--data-size", type=int)
    m.add_argument("--max-chunk-size", type=int)
    m.add_argument("--max-round", type=int)
    m.add_argument("--min-workers", type=int,
                   help="start round 0 once this many workers joined (default: all); the others join later and "
                        "every worker gets a re-InitWorkers with the new peer map (SPEC:141-170)")
    m.add_argument("--max-lag", type=int)
    m.add_argument("--th-allreduce", type=float)
    m.add_argument("--th-reduce", type=float)
    m.add_argument("--th-complete", type=float)
    m.add_argument("--transport", choices=["auto", "rccl", "tcp", "ipc_p2p", "onesided"],
                   help="GPU data plane the master hands out: RCCL (auto/rccl), ipc_p2p = mailboxes in mapped "
                        "peer memory (no RCCL; several workers may share one GPU), or onesided = threshold rounds "
                        "as stores into mapped peer windows (workers --transport onesided; GPU or CPU)")
    m.set_defaults(fn=_master)

    w = sub.add_parser("worker", help="run one AllreduceWorker (one per GPU)")
    w.add_argument("pos", nargs="*", type=int, help="[port] [dataSize]")
    w.add_argument("--config")
    w.add_argument("--port", type=int)
    w.add_argument("--host", help="address this worker listens on and announces to the master (multi-machine: "
                                  "this machine's IP; default 127.0.0.1)")
    w.add_argument("--data-size", type=int)
    w.add_argument("--master", help="host:port of the master")
    w.add_argument("--checkpoint", type=int)
    w.add_argument("--assert-multiple", type=int, default=0)
    w.add_argument("--device", help="cpu | cuda | cuda:N | auto")
    w.add_argument("--dtype", default="float32")
    w.add_argument("--transport", choices=["auto", "stream", "reactive", "outbox", "onesided"], default="auto",
                   help="GPU data path: stream (scheduled RCCL steps) or reactive (per-peer streams, straggler-"
                        "tolerant); outbox = messages through the control plane (CPU); onesided = stores into "
                        "mapped peer windows, fast workers never wait (master --transport onesided)")
    w.set_defaults(fn=_worker)

    d = sub.add_parser("demo", help="master + N CPU workers on localhost")
    d.add_argument("--port", type=int, default=2551)
    d.add_argument("--workers", type=int, default=2)
    d.add_argument("--data-size", type=int, default=10)
    d.add_argument("--max-chunk-size", type=int, default=2)
    d.add_argument("--max-round", type=int, default=100)
    d.add_argument("--max-lag", type=int, default=1)
    d.add_argument("--th-reduce", type=float, default=1.0)
    d.add_argument("--th-complete", type=float, default=1.0)
    d.add_argument("--checkpoint", type=int, default=10)
    d.add_argument("--assert-multiple", type=int, default=0)
    d.add_argument("--timeout", type=float, default=300.0)
    d.set_defaults(fn=_demo)

    i = sub.add_parser("info", help="show native build / device info")
    i.set_defaults(fn=_info)

    a = p.parse_args(argv)
    logging.basicConfig(level=getattr(logging, a.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
