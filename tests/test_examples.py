"""The examples stay runnable: examples/mlp_sgd.py (BASELINE config 5) on two
CPU processes (gloo), a few tiny steps; one JSON line whose loss fell."""
import json
import os
import subprocess
import sys

from test_onesided_cpu import ROOT, _free_port


def test_mlp_sgd_example_on_cpu_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "examples", "mlp_sgd.py"), "--cpu",
           "--steps", "4", "--warmup", "1", "--d-in", "64", "--hidden", "128", "--classes", "10", "--batch", "16"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["loss_last"] < d["loss_first"], d
