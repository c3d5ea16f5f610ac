"""The whole DP-SGD step in one HIP graph: forward,
backward, the one-sided allreduce (its call id / round / decisions are
device-resident, its launch arguments fixed) and the fused average + SGD
update, replayed as one graph on 4 processes sharing the card; and the
same on the exact ipc lane, whose round id then lives in device memory
(``ThresholdAllreduce.capturable()``).  20 steps on
the same batches as the eager step: parameters and losses bitwise equal
(thresholds 1: every sum is the fp32 ascending-source order)."""
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("lane,dtype", [("onesided", "bf16"), ("onesided", "fp32"), ("ipc", "bf16")])
def test_fully_graphed_step_matches_eager(lane, dtype):
    n = 4
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               os.path.join(ROOT, "tests", "graph_ranks.py"), "--out-dir", out, "--dtype", dtype, "--lane", lane]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        rows = [torch.load(os.path.join(out, f"rank{i}.pt"), weights_only=True) for i in range(n)]
    for d in rows:
        assert d["replays"] == 20 and d["calls"] == 20 and d["error"] == 0 and d["forced"] == 0
        if lane == "onesided":
            # exact rounds: round id == call id; the eager call after the
            # graph replays is the last call and its status record is found
            assert d["eager_after_exact"] and d["eager_after_call"] == d["calls_total"] - 1, d
            assert d["eager_after_round"] == d["eager_after_call"], d
        assert torch.equal(d["eager"], d["graphed"])
        assert torch.equal(d["eager_losses"], d["graph_losses"])
    for d in rows[1:]:
        assert torch.equal(d["graphed"], rows[0]["graphed"])  # every rank holds the same model
