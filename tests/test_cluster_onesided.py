"""The reference's actor API on the one-sided threshold lane, with master
pacing (AllreduceMaster.scala:54-63 + AllreduceWorker.scala:7-8, 197-210):
a master process and 4 worker processes (``--transport onesided``),
thAllreduce = thReduce = thComplete = 0.75, maxLag 1, one worker's data
source sleeping 50 ms per round.  The fast workers keep their pace: their
median round stays within 2x of the same job without the straggler, the
straggler catches up by skipping rounds (force-completed, W:100-106), and
every sink sees chunks whose value encodes a contributor set of the size of
its count.  CPU processes here (shared-memory windows, the GPU kernels'
protocol functions); tests/test_cluster_onesided_gpu.py runs the same job
with every worker on the box's GPU."""
import glob
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_job(device="cpu", delay_ms=0.0, rounds=64, size=1 << 14, chunk=1 << 10, workers=4, timeout=240,
            log_dir=None, die_after=-1, env=None):
    port = _port()
    base = [sys.executable, "-m", "akka_allreduce_amd", "--log-level", "WARNING"]
    with tempfile.TemporaryDirectory() as out:
        logs = log_dir or out
        os.makedirs(logs, exist_ok=True)
        # stderr into files, never a pipe nobody reads while waiting (a full
        # pipe would block a chatty process)
        mlog = open(os.path.join(logs, f"master_d{int(delay_ms)}.log"), "w")
        master = subprocess.Popen(base + ["master", "--port", str(port), "--workers", str(workers), "--data-size",
                                          str(size), "--max-chunk-size", str(chunk), "--max-round", str(rounds - 1),
                                          "--max-lag", "1", "--th-allreduce", "0.75", "--th-reduce", "0.75",
                                          "--th-complete", "0.75", "--transport", "onesided"],
                                  cwd=ROOT, stdout=subprocess.DEVNULL, stderr=mlog, env=env)
        t_end = time.time() + 60
        while time.time() < t_end:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                break
            except OSError:
                time.sleep(0.1)
        procs, wlogs = [], []
        for i in range(workers):
            d = delay_ms if i == workers - 1 else 0.0
            wlogs.append(os.path.join(logs, f"worker{i}_d{int(delay_ms)}.log"))
            extra = ["--die-after", str(die_after)] if die_after >= 0 and i == workers - 1 else []
            procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "cluster_onesided_ranks.py"),
                                           "--master", f"127.0.0.1:{port}", "--size", str(size), "--device", device,
                                           "--delay-ms", str(d), "--out-dir", out, "--timeout-s", str(timeout - 30),
                                           *extra],
                                          cwd=ROOT, stdout=subprocess.DEVNULL, stderr=open(wlogs[-1], "w"), env=env))
            if i < workers - 1:
                time.sleep(0.3)  # join order = ids: the straggler joins last (id 3)
        errs = []
        try:
            for p, lg in zip(procs, wlogs):
                try:
                    p.wait(timeout=timeout)
                finally:
                    errs.append(open(lg).read()[-2000:])
            master.wait(timeout=30)
        finally:
            for p in procs + [master]:
                if p.poll() is None:
                    p.kill()
                    p.wait()
            mlog.close()
        rows = [json.load(open(f)) for f in glob.glob(os.path.join(out, "worker*.json"))]
    return rows, errs


def fast_median_ms(rows):
    meds = []
    for r in rows:
        if r["straggler"]:
            continue
        t = [x["t"] for x in r["records"]]
        gaps = [(b - a) * 1e3 for a, b in zip(t, t[1:])]
        tail = gaps[len(gaps) // 2:]
        meds.append(statistics.median(tail))
    return max(meds)


def check_job(device, rounds=64, slack_ms=2.0, **kw):
    import os as _os

    kw.setdefault("log_dir", _os.environ.get("AKKA_TEST_LOGS") or None)
    base, e0 = run_job(device, 0.0, rounds, **kw)
    assert len(base) == 4, e0
    strag, e1 = run_job(device, 50.0, rounds, **kw)
    assert len(strag) == 4, e1
    for rows in (base, strag):
        for r in rows:
            assert r["finished"] and not r["errors"], r["errors"]
            assert all(x["bad"] == 0 for x in r["records"]), r["id"]
            rs = [x["round"] for x in r["records"]]
            assert rs == sorted(rs) and len(set(rs)) == len(rs), rs[:20]
    for r in base:
        assert [x["round"] for x in r["records"]] == list(range(rounds))
    b, s = fast_median_ms(base), fast_median_ms(strag)
    assert s <= 2 * b + slack_ms, (b, s)
    st = [r for r in strag if r["straggler"]][0]
    assert st["forced_rounds"] > 0 and len(st["records"]) < rounds + st["forced_rounds"] + 1
    fast = [r for r in strag if not r["straggler"]]
    for r in fast:
        assert r["records"][-1]["round"] == rounds - 1
        assert min(x["mean_count"] for x in r["records"]) >= 2.0  # 3 of 4 contributors at least on most chunks
    return b, s


def test_cluster_onesided_master_pacing_cpu():
    check_job("cpu")


def test_cluster_onesided_worker_dies():
    """A worker process exits abruptly after round 10 (no Shutdown, no
    retire).  The master notices (WorkerTerminated, M:46-52), paces the
    remaining rounds on the live count, the survivors mark the rank dead in
    their lanes and serve every round to maxRound with consistent contributor
    sets -- the dead rank's block 0 with count 0 (C1e)."""
    env = dict(os.environ, AKKA_CLUSTER_UNREACHABLE_AFTER_S="2", AKKA_CLUSTER_HEARTBEAT_INTERVAL_S="0.25")
    rows, errs = run_job("cpu", 0.0, 48, die_after=10, env=env)
    assert len(rows) == 3, errs  # the dead worker writes no record
    for r in rows:
        assert r["finished"] and not r["errors"], (r["errors"], errs)
        assert all(x["bad"] == 0 for x in r["records"]), r["id"]
        rs = [x["round"] for x in r["records"]]
        assert rs == sorted(rs) and rs[-1] == 47, rs[-5:]
        # rounds after the death: 3 contributors at most per chunk
        late = [x for x in r["records"] if x["round"] >= 20]
        assert late and max(x["mean_count"] for x in late) <= 3.0, late[:3]
