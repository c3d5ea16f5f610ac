#!/usr/bin/env python3
"""The five BASELINE.json configurations as runnable commands.

  1  master + 2 workers, dataSize 10, chunk 2 (CPU, README demo)
  2  exact allreduce, 256 MB fp32, 4 MB chunks          (= bench.py defaults)
  3  bf16, 1 GB buffer, chunk sized to a per-link share (bench.py --dtype bfloat16 --size-mb 1024)
  4  thresholds 0.75/0.75, maxLag 1, one induced straggler
  5  2-layer MLP DP-SGD with gradient allreduce         (examples/mlp_sgd.py)

``python bench/configs.py N`` prints the command for config N at the current
world size (use under torch.distributed.run for N>1 GPUs);
``python bench/configs.py N --run`` executes it.

Config 4 runs on the reactive transport (per-peer streams + two-rank RCCL
communicators, event-polled arrivals): with thresholds 0.75 the fast ranks
complete rounds without waiting for the straggler.  On the scheduled
transport every rank still exchanges every chunk (RCCL p2p is a rendezvous),
so a straggler delays everyone and the thresholds only decide which
contributions are summed.  ``bench.py`` (default invocation) also times
configs 3 and 5 after the headline and reports them under ``extra_configs``.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def command(n: int, world: int) -> list[str]:
    if n == 1:
        return [PY, "-m", "akka_allreduce_amd", "demo", "--workers", "2", "--data-size", "10", "--max-chunk-size", "2",
                "--max-round", "100", "--max-lag", "1", "--th-complete", "0.8", "--checkpoint", "50"]
    if n == 2:
        return [PY, os.path.join(ROOT, "bench.py"), "--gpus", str(world)]
    if n == 3:
        # 1 GiB bf16: each rank's block is 1/N of it; 8 MiB chunks keep 8-64 chunks in flight per link
        return [PY, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dtype", "bfloat16", "--size-mb", "1024",
                "--chunk-mb", "8"]
    if n == 4:
        return [PY, os.path.join(ROOT, "bench", "straggler.py"), "--th-reduce", "0.75", "--th-complete", "0.75",
                "--max-lag", "1", "--transport", "reactive"]
    if n == 5:
        return [PY, os.path.join(ROOT, "examples", "mlp_sgd.py")]
    raise SystemExit(f"unknown config {n}")


if __name__ == "__main__":
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cmd = command(cfg, int(os.environ.get("WORLD_SIZE", "1")))
    if "--run" in sys.argv:
        sys.exit(subprocess.call(cmd, cwd=ROOT))
    print(" ".join(cmd))
