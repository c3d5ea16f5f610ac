"""Master/worker cluster runtime (TCP control + data plane on CPU).

* README demo (BASELINE config 1): master + 2 workers, dataSize 10, chunk 2.
* scripts config: 4 workers, dataSize 778, chunk 3, maxLag 3, exact (x4).
* failure detection: a worker dies mid-run; with thresholds < 1 the survivors
  keep completing rounds and the master (live-count pacing) reaches maxRound.
* separate OS processes via the CLI (`python -m akka_allreduce_amd demo`).
"""
import os
import subprocess
import sys
import time

import pytest

from akka_allreduce_amd.config import DataConfig, ThresholdConfig, WorkerConfig
from akka_allreduce_amd.parallel.cluster import start_master, start_worker

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_cluster(n, size, chunk, rounds, max_lag=1, th=(1.0, 1.0, 1.0), assert_multiple=None, checkpoint=5):
    m = start_master(ThresholdConfig(*th), DataConfig(size, chunk, rounds), WorkerConfig(n, max_lag), port=0,
                     transport="tcp", unreachable_after_s=30.0)
    am = n if assert_multiple is None else assert_multiple
    ws = [start_worker(m.address, size, checkpoint=checkpoint, assert_multiple=am, printer=lambda *_: None)
          for _ in range(n)]
    try:
        assert m.wait(60), f"master stuck at round {m.master.round}"
        for w in ws:
            assert w.wait(10)
        return m, ws
    finally:
        m.stop()
        for w in ws:
            w.stop()


def test_readme_demo_two_workers():
    m, ws = _run_cluster(2, 10, 2, 40)
    assert m.master.round == 40
    for w in ws:
        assert w.worker.dataSink.failures == 0
        assert w.worker.dataSink.rounds >= 41


def test_scripts_config_four_workers_exact():
    # scripts/testAllreduceMaster.sc: 4 workers, 778 floats, chunk 3, maxLag 3, thresholds 1 (maxRound cut to 30)
    m, ws = _run_cluster(4, 778, 3, 30, max_lag=3, checkpoint=10)
    for w in ws:
        assert w.worker.dataSink.failures == 0
    assert sorted(w.worker.id for w in ws) == [0, 1, 2, 3]


def test_node_metrics_on_heartbeats():
    """Cluster metrics (CONF:26-34): workers attach a node sample to heartbeats; master keeps the latest."""
    from akka_allreduce_amd.messages import Heartbeat
    from akka_allreduce_amd.parallel.wire import decode, encode
    from akka_allreduce_amd.utils.node_metrics import sample

    s = sample(gpus=False)
    assert s["mem_total_mb"] > 0 and s["mem_used_mb"] >= 0 and "cpu_pct" in s
    hb = decode(encode(Heartbeat(3, 7, s), lambda r: None)[4:], lambda a: None)  # [4:]: frame header
    assert (hb.srcId, hb.round, hb.metrics) == (3, 7, s)
    assert decode(encode(Heartbeat(1, 2), lambda r: None)[4:], lambda a: None).metrics is None

    # (enough rounds to outlast several heartbeats: the job must still run
    # when the first samples go out -- 200 rounds take ~0.1 s now)
    size, rounds = 100, 1_000_000
    m = start_master(ThresholdConfig(1.0, 1.0, 1.0), DataConfig(size, 10, rounds), WorkerConfig(2, 1), port=0,
                     transport="tcp", unreachable_after_s=30.0, heartbeat_interval_s=0.1)
    ws = [start_worker(m.address, size, checkpoint=1000, printer=lambda *_: None, heartbeat_interval_s=0.1,
                       metrics_interval_s=0.05) for _ in range(2)]
    try:
        t0 = time.time()
        while len(m.node_metrics) < 2 and time.time() - t0 < 20:
            time.sleep(0.05)
        assert sorted(m.node_metrics) == [0, 1]
        assert all(v["mem_total_mb"] > 0 for v in m.node_metrics.values())
    finally:
        m.stop()
        for w in ws:
            w.stop()


def test_worker_death_with_thresholds():
    """A worker dies mid-run (stops heartbeating and serving): the master's
    failure detector declares it down (M:46-52) and the survivors finish.
    Round 2's rare RuntimeError here was Node.stop() iterating the connection
    map while the victim's heartbeat thread inserted a connection into it
    (fixed: every access holds the node's connection lock).  The unreachable
    bound is 3 s with 0.1 s heartbeats, so a loaded CI machine does not
    declare a live worker dead."""
    n, size, chunk, rounds = 3, 300, 10, 400
    # thReduce .66 -> 1 of 3 copies, thComplete .3 of 30 chunks, thAllreduce .6 of live workers
    m = start_master(ThresholdConfig(0.6, 0.66, 0.3), DataConfig(size, chunk, rounds), WorkerConfig(n, 2), port=0,
                     transport="tcp", unreachable_after_s=3.0, heartbeat_interval_s=0.1)
    ws = [start_worker(m.address, size, checkpoint=1000, printer=lambda *_: None, heartbeat_interval_s=0.1)
          for _ in range(n)]
    try:
        t0 = time.time()
        while m.master.round < 5 and time.time() - t0 < 60:
            time.sleep(0.02)
        assert m.master.round >= 5
        victim = ws[2]
        victim.stop()  # dies: stops heartbeating and serving
        assert m.wait(120), f"stalled at round {m.master.round} with {len(m.master.workers)} workers"
        assert len(m.master.workers) == n - 1
    finally:
        m.stop()
        for w in ws:
            w.stop()


def test_cli_demo_processes():
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    port = 26000 + (os.getpid() % 3000)
    r = subprocess.run([sys.executable, "-m", "akka_allreduce_amd", "--log-level", "WARNING", "demo", "--port",
                        str(port), "--workers", "2", "--data-size", "10", "--max-chunk-size", "2", "--max-round", "25",
                        "--checkpoint", "5", "--assert-multiple", "2", "--timeout", "120"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "failures=0" in r.stdout


def test_node_poller_drives_progress_between_messages():
    """The dispatcher thread runs the poller while it reports pending work
    (the reactive GPU transport's in-flight transfers) and blocks on the
    mailbox once it returns None."""
    import threading
    import time

    from akka_allreduce_amd.parallel.actors import Node

    got = []
    pending = {"n": 5}
    polled = threading.Event()

    class A:
        def receive(self, msg):
            got.append(msg)

    node = Node("127.0.0.1", 0, name="p")

    def poller():
        if pending["n"] == 0:
            polled.set()
            return None
        pending["n"] -= 1
        return pending["n"] % 2 == 0

    node.poller = poller
    node.start(A())
    try:
        node.send(node.address, "hello")
        assert polled.wait(5)
        node.send(node.address, "again")
        t0 = time.time()
        while len(got) < 2 and time.time() - t0 < 5:
            time.sleep(0.01)
        assert got == ["hello", "again"]
        assert pending["n"] == 0
    finally:
        node.stop()


def test_worker_process_rejects_gpu_transports_on_cpu():
    from akka_allreduce_amd.parallel.cluster import WorkerProcess

    with pytest.raises(ValueError):
        WorkerProcess("127.0.0.1:1", None, None, device="cpu", transport="reactive")


def test_reference_startup_entry_points():
    """AllreduceMaster.startUp / AllreduceWorker.startUp with the reference's
    signatures (M:138-144, W:348-362) run the README demo shape."""
    from akka_allreduce_amd import AllreduceMaster, AllreduceWorker

    m = AllreduceMaster.startUp(0, ThresholdConfig(1.0, 1.0, 1.0), DataConfig(10, 2, 20), WorkerConfig(2, 1),
                                transport="tcp")
    ws = [AllreduceWorker.startUp(0, 10, 5, 2, master=m.address, printer=lambda *a: None) for _ in range(2)]
    try:
        assert m.wait(60)
        for w in ws:
            assert w.wait(30)
            assert w.worker.dataSink.failures == 0 and w.worker.dataSink.rounds >= 20
    finally:
        m.stop()
        for w in ws:
            w.stop()
