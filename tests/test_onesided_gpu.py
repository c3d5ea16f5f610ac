"""The one-sided threshold lane on the GPU: every rank is a process on the
box's one MI355X, windows are fine-grained HBM mapped through IPC handles,
the rounds are the gfx950 kernels of csrc/kernels/onesided.hip (cross-XCD
hand-offs; the same code crosses xGMI on a node).  Same scenarios as
tests/test_onesided_cpu.py, whose protocol functions these kernels share."""
import pytest

from test_onesided_cpu import assert_fast_rank_did_not_wait, run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,size,chunk,dtype", [
    (2, 1 << 20, 1 << 16, "float32"),
    (3, 1_000_003, 40_000, "float32"),    # uneven blocks: scalar paths, short last chunks
    (4, 1 << 22, 1 << 18, "bfloat16"),
    (2, 10, 2, "float32"),                # the reference's README demo geometry
    (4, 1 << 24, 1 << 20, "float32"),     # 64 MiB, 4 MiB chunks, 16 parts each (BASELINE config 4's shape)
    (8, 1 << 22, 1 << 17, "float32"),     # a node's rank count: the N=8 masked-sum kernel
    (8, 1 << 22, 1 << 17, "bfloat16"),
])
@pytest.mark.parametrize("handoff", ["lite", "fenced"])
def test_onesided_gpu_exact_rounds(n, size, chunk, dtype, handoff):
    """Both hand-off modes (write-through + drain; plain stores behind
    system release / acquire): bitwise the fp32 sum, counts N."""
    r, rows = run_ranks(n, "--mode", "exact", "--size", str(size), "--chunk", str(chunk), "--dtype", dtype,
                        "--rounds", "4", "--timeout-s", "10", "--handoff", handoff, device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["info"]["backend"] == "gpu" and d["info"]["handoff"] == handoff
        assert d["exact"] == [True] * 4, d
        assert d["rounds"] == list(range(4)), d
        assert d["error"] == 0 and d["stats"]["missing_chunks"] == 0, d["stats"]


@pytest.mark.parametrize("n,size,chunk,dtype,wo", [
    (2, 1 << 20, 1 << 16, "float32", True),
    (4, 1 << 24, 1 << 20, "float32", True),    # 64 MiB, 4 MiB chunks
    (8, 1 << 22, 1 << 17, "bfloat16", True),
    (3, 1_000_003, 40_000, "float32", False),  # a block's bytes not a 16-B multiple: the classic copy
])
@pytest.mark.parametrize("handoff", ["lite", "fenced"])
def test_onesided_gpu_window_output(n, size, chunk, dtype, wo, handoff):
    """Exact rounds whose output is the gather row of the call in the rank's
    own window (no copy): bitwise the fp32 sum, counts N, rounds in order,
    each output the row of its call id (rows cycle)."""
    r, rows = run_ranks(n, "--mode", "exact", "--size", str(size), "--chunk", str(chunk), "--dtype", dtype,
                        "--rounds", "5", "--timeout-s", "10", "--window-output", "--handoff", handoff,
                        device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["info"]["window_output"] is wo, d["info"]
        assert d["exact"] == [True] * 5 and d["rounds"] == list(range(5)), d
        assert d.get("in_window", [True] * 5 if wo else None) == ([True] * 5 if wo else None), d
        assert d["error"] == 0 and d["stats"]["missing_chunks"] == 0, d["stats"]
        if wo:  # a kept row holds its lane: still the last sum after the object went, freed with the row
            assert d["kept_row_alive"] and d["kept_row_exact"] and d["row_dropped_frees_lane"], d


def test_onesided_gpu_exact_rounds_async():
    """async_op=True: the round runs on the lane's side stream behind the
    caller's stream (the input's host-to-device copy); wait() joins it."""
    r, rows = run_ranks(4, "--mode", "exact", "--size", str(1 << 22), "--chunk", str(1 << 18), "--rounds", "4",
                        "--async-op", "--timeout-s", "10", device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["exact"] == [True] * 4 and d["error"] == 0, d


def test_onesided_gpu_timeline_stamps():
    """AKKA_OS_TIMELINE=1: every workgroup of the last call stamped [entry,
    round known, role done] in order (bench/onesided_timeline.py's input)."""
    r, rows = run_ranks(2, "--mode", "exact", "--size", str(1 << 20), "--chunk", str(1 << 16), "--rounds", "2",
                        "--timeline", "--timeout-s", "10", device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        t = d["timeline"]
        assert d["exact"] == [True] * 2 and t["words"] >= 3 * t["grid"] and t["ordered"] and t["span_ticks"] > 0, t


@pytest.mark.parametrize("handoff", ["lite", "fenced"])
def test_onesided_gpu_straggler_steady_state(handoff):
    """N=4 on the card, 0.75 / 0.75, maxLag 1, rank 3 sleeps 50 ms per call,
    64 rounds: fast ranks' calls complete on the threshold with the
    straggler's copy in few of their chunks (assert_fast_rank_did_not_wait),
    contributor sets consistent with counts, straggler's pushes dropped --
    in both hand-off modes."""
    r, rows = run_ranks(4, "--mode", "straggler", "--straggler", "3", "--rounds", "64", "--compute-ms", "2",
                        "--delay-ms", "50", "--size", str(1 << 22), "--chunk", str(1 << 18), "--timeout-s", "10",
                        "--handoff", handoff, device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["error"] == 0, d["stats"]
        for ph in ("no_straggler", "straggler"):
            assert d[ph]["bad_chunks"] == 0 and d[ph]["own_block_has_me"], (d["rank"], ph, d[ph]["bad_detail"], d[ph]["stats"])
    for d in rows[:3]:
        assert_fast_rank_did_not_wait(d, delay_ms=50.0)
    s = rows[3]["stats"]
    assert s["skipped_rounds"] > 0 and s["scatter_outdated"] + s["gather_outdated"] > 0, s


def test_onesided_gpu_straggler_killed_mid_run():
    """The straggler process exits abruptly (os._exit: no retire, no
    teardown) after 3 calls of the straggler phase while the survivors keep
    storing into its (still mapped) window: they complete every round to the
    end, contributor sets consistent, no timeout."""
    r, rows = run_ranks(4, "--mode", "straggler", "--straggler", "3", "--rounds", "48", "--compute-ms", "2",
                        "--delay-ms", "30", "--kill-after", "3", "--size", str(1 << 20), "--chunk", str(1 << 16),
                        "--timeout-s", "10", device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert rows[3]["killed_after"] == 3
    for d in rows[:3]:
        assert d["error"] == 0 and d["straggler"]["bad_chunks"] == 0, d["stats"]
        assert d["straggler"]["rounds"][-1] >= 95 and d["stats"]["timeouts"] == 0


@pytest.mark.parametrize("n,th,max_lag,dtype", [(4, 0.75, 1, "float32"), (8, 0.5, 2, "bfloat16"),
                                                (3, 0.67, 1, "float32"), (4, 1.0, 1, "float32")])
@pytest.mark.parametrize("handoff", ["lite", "fenced"])
def test_onesided_gpu_chaos_jitter(n, th, max_lag, dtype, handoff):
    """Every rank waits a random 0-2 ms before each call, 200 rounds, 16 MiB
    (fp32) with 1 MiB chunks: arrival orders, lags, catch-ups and overwrite
    conflicts vary from round to round across the card's XCDs.  Every output
    chunk of every call is one contributor set matching its count."""
    r, rows = run_ranks(n, "--mode", "chaos", "--th", str(th), "--max-lag", str(max_lag), "--rounds", "200",
                        "--jitter-ms", "2", "--size", str(1 << 22), "--chunk", str(1 << 18), "--dtype", dtype,
                        "--timeout-s", "10", "--handoff", handoff, device="cuda", timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        c = d["chaos"]
        assert c["bad_chunks"] == 0, (d["rank"], c["bad_detail"], c["stats"])
        assert d["error"] == 0 and c["stats"]["timeouts"] == 0, c["stats"]
        assert c["rounds"][-1] >= 199, c["rounds"][-5:]
        if th == 1.0:  # exact thresholds: whatever the timing, every round is complete
            assert c["calls_with_partial_chunks"] == 0 and c["rounds"] == list(range(200)), c["stats"]


def test_onesided_gpu_dead_peer_marked():
    """GPU twin of tests/test_onesided_cpu.py::test_onesided_dead_peer_marked:
    a rank vanishes without retiring, the survivors mark it dead and keep
    completing exact rounds over the live ranks, no wait times out."""
    r, rows = run_ranks(4, "--mode", "dead", "--kill-after", "3", "--rounds", "10", "--size", str(1 << 20),
                        "--chunk", str(1 << 16), "--timeout-s", "10", device="cuda", timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows[:3]:
        dd = d["dead"]
        assert dd["before"] == [0, 1, 2] and dd["after"] == list(range(3, 13)), dd
        assert dd["bad_chunks"] == 0 and d["error"] == 0 and d["stats"]["timeouts"] == 0, (dd, d["stats"])
