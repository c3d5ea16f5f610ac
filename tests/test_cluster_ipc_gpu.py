"""The reference's architecture end to end on the GPU with several worker
PROCESSES: a master (this process, CPU only) paces rounds and hands out the
data plane in InitWorkers; three worker processes (the CLI, `python -m
akka_allreduce_amd worker`) share the box's one MI355X and move their chunks
through mailboxes in each other's mapped memory (ipc_p2p: no RCCL, whose
communicators refuse two ranks on one device).  The window handles meet in a
store hosted by the master.  The demo sink checks every round
(output == 3 x input, counts == 3) like the reference's assertMultiple
(W:337-340); the master runs to maxRound and shuts the workers down."""
import os
import subprocess
import sys

import pytest

from akka_allreduce_amd.config import DataConfig, ThresholdConfig, WorkerConfig
from akka_allreduce_amd.parallel.cluster import start_master

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("transport,size,chunk", [("stream", 778, 3), ("stream", 1 << 20, 1 << 15),
                                                  ("reactive", 1 << 18, 1 << 14)])
def test_master_with_three_gpu_worker_processes(transport, size, chunk):
    n, rounds = 3, 20
    m = start_master(ThresholdConfig(1.0, 1.0, 1.0), DataConfig(size, chunk, rounds), WorkerConfig(n, 2), port=0,
                     transport="ipc_p2p", unreachable_after_s=60.0)
    env = dict(os.environ, AKKA_SHARE_GPU="1", GPU_MAX_HW_QUEUES="8")
    procs = [subprocess.Popen([sys.executable, "-m", "akka_allreduce_amd", "worker", "--master", m.address,
                               "--data-size", str(size), "--checkpoint", "5", "--assert-multiple", str(n),
                               "--device", "cuda:0", "--transport", transport],
                              cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for _ in range(n)]
    try:
        assert m.wait(150), f"master stuck at round {m.master.round}"
        outs = [p.communicate(timeout=60)[0] for p in procs]
    finally:
        m.stop()
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
        line = [ln for ln in out.splitlines() if ln.startswith("worker ")][-1]
        assert "failures=0" in line, line
        assert int(line.split("rounds=")[1].split()[0]) >= rounds - 2, line
