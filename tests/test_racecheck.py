"""Stream race checking on the CPU simulator (csrc/engine/racecheck.h).

With AKKA_RACECHECK=1 every simulated rank's device tracks happens-before over
its streams and events (vector clocks) and the bytes each op reads and writes.
Each worker also gets a modelled caller stream: the producer of its inputs,
the allocator of its outputs and the reader of its results.  The tests model
the caller's side of a round explicitly:

  * it wrote the input on its stream before the call;
  * the output and counts memory it hands over may still be written by
    earlier work on its stream (the caching allocator recycles freed blocks in
    that stream's order) -- declared as a pending write right after allocation;
  * it reads the results on its stream after the call.

Every lane and threshold schedule must be race-free under that contract; the
checker must flag the round-2 counts-fill race when it is re-injected
(AKKA_FAULT_SKIP_OUTPUT_WAIT=1) and a caller that reads results off-stream.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {root!r})
import torch
from akka_allreduce_amd.parallel.sim import SimCluster

cfg = json.loads(sys.argv[1])
n, S, C = cfg["n"], cfg["S"], cfg["C"]
c = SimCluster(n, S, C, lane=cfg["lane"], collectives=cfg["collectives"], max_lag=cfg.get("max_lag", 2),
               th_reduce=cfg.get("th", 1.0), th_complete=cfg.get("th", 1.0))
assert all(w.host_stream for w in c.workers), "race checking is not on"

def hook(w):
    orig = w._new_output_buffers
    def hooked(r):
        out, counts = orig(r)
        # recycled memory: earlier caller work on its stream still writes it
        w._core.declare_access(w.host_stream, out.data_ptr(), out.numel() * out.element_size(), True,
                               "caller.pending_write")
        w._core.declare_access(w.host_stream, counts.data_ptr(), counts.numel() * 4, True, "caller.pending_write")
        return out, counts
    w._new_output_buffers = hooked

for w in c.workers:
    hook(w)
off = None
for rnd in range(cfg.get("rounds", 3)):
    xs = [torch.randn(S) for _ in range(n)]
    for w, x in zip(c.workers, xs):
        w._core.declare_access(w.host_stream, x.data_ptr(), x.numel() * 4, True, "caller.input_write")
    outs = [w.allreduce(x) for w, x in zip(c.workers, xs)]
    c.run()
    for w, o in zip(c.workers, outs):
        if o is None:
            continue
        if cfg.get("offstream_read"):
            off = off or w._core.create_stream()
            w._core.declare_access(off, o.data.data_ptr(), o.data.numel() * 4, False, "caller.offstream_read")
        else:
            w._core.declare_access(w.host_stream, o.data.data_ptr(), o.data.numel() * 4, False, "caller.read")
            pc = o.counts_per_chunk
            w._core.declare_access(w.host_stream, pc.data_ptr(), pc.numel() * 4, False, "caller.read")
    c.run()
    if cfg.get("th", 1.0) >= 1.0:
        want = sum(xs)
        for o in outs:
            assert torch.allclose(o.data, want, atol=1e-4)
            assert bool((o.counts_per_chunk == n).all())
st = c.workers[0].state()["link"]
print(json.dumps({{"races": [w._core.race_count() for w in c.workers], "reports": c.race_reports()[:8],
                  "collective_rounds": st.get("collective_rounds"), "exact_step_rounds": st.get("exact_step_rounds")}}))
'''


def _run(cfg, **env):
    import json

    e = dict(os.environ)
    e["AKKA_RACECHECK"] = "1"
    e.update(env)
    r = subprocess.run([sys.executable, "-c", _SCRIPT.format(root=ROOT), json.dumps(cfg)], capture_output=True,
                       text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("lane,collectives", [("collective", True), ("collective", False), ("p2p", False)])
@pytest.mark.parametrize("n,S,C", [(2, 1000, 64), (4, 4096, 256), (8, 8192, 128)])
def test_exact_lanes_are_race_free(lane, collectives, n, S, C):
    if lane == "collective" and collectives and S % n:
        pytest.skip("native collectives need an even split")
    d = _run({"n": n, "S": S, "C": C, "lane": lane, "collectives": collectives})
    assert sum(d["races"]) == 0, d["reports"]
    if lane == "collective":
        assert d["collective_rounds"] == 3
    else:
        assert d["exact_step_rounds"] == 3


@pytest.mark.parametrize("n,S,C,th", [(3, 63 * 4, 4, 0.67), (4, 64 * 4, 4, 0.75)])
def test_threshold_schedule_is_race_free(n, S, C, th):
    d = _run({"n": n, "S": S, "C": C, "lane": "p2p", "collectives": False, "th": th})
    assert sum(d["races"]) == 0, d["reports"]


def test_detects_the_counts_fill_race_when_reinjected():
    """The round-2 bug: the exact round's counts fill did not wait for the
    caller's hand-over point.  Re-injected, the checker names it on every rank
    (fill vs the caller's pending write).  (Since round 5 an exact bulk round
    fills its counts on the comm stream, behind that stream's wait for the
    hand-over, which the fault now skips.)"""
    d = _run({"n": 4, "S": 4096, "C": 256, "lane": "collective", "collectives": True},
             AKKA_FAULT_SKIP_OUTPUT_WAIT="1")
    assert all(r > 0 for r in d["races"]), d
    assert any("fill_i32" in m and "caller.pending_write" in m for m in d["reports"]), d["reports"]


def test_detects_a_caller_reading_results_off_stream():
    d = _run({"n": 2, "S": 1000, "C": 64, "lane": "p2p", "collectives": False, "offstream_read": True})
    assert sum(d["races"]) > 0
    assert any("caller.offstream_read" in m for m in d["reports"]), d["reports"]


_REACTIVE = r'''
import json, sys
sys.path.insert(0, {root!r})
import torch
from akka_allreduce_amd.parallel.sim import ReactiveSimCluster

cfg = json.loads(sys.argv[1])
n, S, C, th, slow = cfg["n"], cfg["S"], cfg["C"], cfg["th"], cfg["slow"]
c = ReactiveSimCluster(n, S, C, th_reduce=th, th_complete=th, max_lag=1, seed=3)
assert all(w.host_stream for w in c.workers), "race checking is not on"
fast = [k for k in range(n) if k != slow]
for r in range(cfg["rounds"]):
    for k in range(n):
        if k == slow and r > 0:
            continue  # frozen after round 0: the others must not wait for it
        x = torch.randn(S)
        w = c.workers[k]
        w._core.declare_access(w.host_stream, x.data_ptr(), x.numel() * 4, True, "caller.input_write")
        c.start(k, x)
    c.run(lambda: all(c.done(k, r) for k in fast), shuffle=True)
    for k in fast:
        w, o = c.workers[k], c.outputs[k][r]
        s = w.host_stream if not cfg.get("offstream_read") else w._core.create_stream()
        w._core.declare_access(s, o.data.data_ptr(), o.data.numel() * 4, False, "caller.read")
c.settle()
print(json.dumps({{"races": [w._core.race_count() for w in c.workers], "reports": c.race_reports()[:8]}}))
'''


def _run_reactive(cfg):
    import json

    e = dict(os.environ)
    e["AKKA_RACECHECK"] = "1"
    r = subprocess.run([sys.executable, "-c", _REACTIVE.format(root=ROOT), json.dumps(cfg)], capture_output=True,
                       text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("th,slow", [(1.0, -1), (0.75, 3)])
def test_reactive_transport_is_race_free(th, slow):
    """Per-peer streams, staged inputs, landing rows, a frozen rank: the
    reactive link's stream/event discipline under shuffled stream order."""
    d = _run_reactive({"n": 4, "S": 1024, "C": 64, "th": th, "slow": slow, "rounds": 4})
    assert sum(d["races"]) == 0, d["reports"]


def test_reactive_offstream_read_is_flagged():
    d = _run_reactive({"n": 3, "S": 600, "C": 64, "th": 1.0, "slow": -1, "rounds": 2, "offstream_read": True})
    assert sum(d["races"]) > 0 and any("caller.read" in m for m in d["reports"]), d


def test_simulator_suites_are_race_free():
    """Every schedule test of the simulator (exact lanes, thresholds, lags,
    uneven geometries, partial membership, reactive fuzzing with frozen and
    dead ranks) re-run with the checker on: the conftest fixture fails any
    test whose clusters report a stream race."""
    e = dict(os.environ)
    e["AKKA_RACECHECK"] = "1"
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_sim_schedule.py"),
                        os.path.join(ROOT, "tests", "test_reactive_sim.py")],
                       capture_output=True, text=True, timeout=900, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "failed" not in r.stdout


def _run_fast(n, lane, mode=""):
    import json
    import socket
    import tempfile

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    e = dict(os.environ)
    e["AKKA_RACECHECK"] = "1"
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(port),
               os.path.join(ROOT, "tests", "race_ranks.py"), "4096", "256", lane, "3", out, mode]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        rows = []
        for i in range(n):
            with open(os.path.join(out, f"rank{i}.json")) as f:
                rows.append(json.load(f))
    return rows


@pytest.mark.parametrize("lane", ["collective", "p2p"])
def test_fast_path_across_processes_is_race_free(lane):
    """ThresholdAllreduce's native fast path (the GPU bench / DP path: caller
    buffers bound in C++) over gloo processes, checked end to end."""
    rows = _run_fast(3, lane)
    for d in rows:
        assert all(d["exact"]) and d["fast_rounds"] == 3, d
        assert d["races"] == 0, d["reports"]


def test_fast_path_offstream_read_is_flagged():
    rows = _run_fast(2, "p2p", "offstream")
    assert all(d["races"] > 0 for d in rows), rows
    assert any("caller.read" in m for d in rows for m in d["reports"])


_UNIT = r'''
import json, sys
sys.path.insert(0, {root!r})
import torch
from akka_allreduce_amd.parallel.sim import SimCluster

c = SimCluster(2, 64, 8)
core = c.workers[0]._core
a, b = core.create_stream(), core.create_stream()
buf = torch.zeros(1024)
p = buf.data_ptr()
res = {{}}
def count():
    return core.race_count()
core.declare_access(a, p, 64, True, "w1"); core.declare_access(a, p, 64, True, "w2")
res["same_stream_ww"] = count()
core.declare_access(a, p + 128, 64, False, "r1"); core.declare_access(b, p + 128, 64, False, "r2")
res["two_streams_rr"] = count()
core.declare_access(b, p, 32, True, "w3")
res["two_streams_ww"] = count()
core.sync_stream(a); core.sync_stream(b)
core.declare_access(a, p, 64, True, "w4")
res["after_host_sync"] = count()
core.declare_access(b, p + 256, 64, True, "w5"); core.declare_access(a, p + 300, 8, False, "r3")
res["partial_overlap_wr"] = count()
print(json.dumps(res))
'''


def test_checker_unit_semantics():
    """Same-stream order, read/read, unordered write/write, host-sync joins,
    partial range overlap."""
    import json

    e = dict(os.environ)
    e["AKKA_RACECHECK"] = "1"
    r = subprocess.run([sys.executable, "-c", _UNIT.format(root=ROOT)], capture_output=True, text=True,
                       timeout=120, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d == {"same_stream_ww": 0, "two_streams_rr": 0, "two_streams_ww": 1, "after_host_sync": 1,
                 "partial_overlap_wr": 2}, d
