"""bench.py's multi-rank flow rehearsed on CPU (gloo), the way the driver
launches N>1: torch.distributed.run, one process per rank, rank 0 prints one
JSON line, every rank exits 0.  Covers the barrier/max-over-ranks timing, the
exactness check across ranks, the comparator group, and the extras deadline
(every rank leaves through it).  The RCCL/xGMI data path itself is covered by
the GPU loopback tests; these numbers are not the metric."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, *extra, env=None, expect_rc=0):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "3", "--warmup", "1", "--size-mb", "0.5", "--chunk-mb", "0.0625",
           "--device", "cpu", *extra]
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=e)
    if expect_rc == 0:
        assert r.returncode == 0, r.stderr[-3000:]
    else:
        assert r.returncode != 0, r.stdout[-3000:]
    # stdout carries exactly the one JSON line (banners of gloo / RCCL and any
    # rank's prints are moved to stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), (r.stdout, r.stderr[-3000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("n,transport", [(2, "stream"), (3, "stream"), (2, "reactive")])
def test_bench_multirank_line(n, transport):
    d = _run(n, "--transport", transport, "--lane-select", "off")
    assert d["n_gpus"] == n and d["steps"] == 3 and d["warmup"] == 1
    assert d["exact"] is True and d["value"] > 0
    assert d["config"]["parallelism"] == f"dp{n}" and d["config"]["transport"] == "gloo-p2p"
    assert abs(d["busbw_GBps"] - d["value"] * 2 * (n - 1) / n) < 1e-2
    assert d["rccl_allreduce_algbw_GBps"] and d["rccl_allreduce_algbw_GBps"] > 0
    # self-proving fields: what the transport itself reports, per rank
    assert d["scaling"] == "strong" and d["preflight"] == "passed"
    assert d["p2p_nranks"] == n and "rccl_nranks" in d and "rccl_version" in d
    assert [r["rank"] for r in d["rank_devices"]] == list(range(n))
    assert all(r["p2p"]["nranks"] == n and r["p2p"]["rank"] == r["rank"] for r in d["rank_devices"])
    assert d["groups_per_round"] > 0 and d["host_us_per_round"] > 0
    # gloo has no native collectives: auto keeps the chunk schedule, and the
    # whole-round lane is measured as the other lane (stream transport only)
    assert d["lane"] == "p2p" and d["lane_is_framework"] is True
    # per-link probe: an N x N matrix per direction (row = source), no diagonal
    lp = d["link_probe"]
    for key in ("push_GBps", "pull_GBps"):
        m = lp[key]
        assert len(m) == n and all(len(row) == n for row in m)
        assert all((m[i][j] is None) == (i == j) for i in range(n) for j in range(n))
        assert all(m[i][j] > 0 for i in range(n) for j in range(n) if i != j)
    assert len(lp["all_peers_push_GBps_per_rank"]) == n and "not a link measurement" in lp["note"]
    if transport == "stream":
        assert d["other_lane"]["lane"] == "collective" and d["other_lane"]["algbw_GBps"] > 0


def test_bench_collective_lane_line():
    d = _run(3, "--lane", "collective")
    assert d["exact"] is True and d["lane"] == "collective" and d["other_lane"]["lane"] == "p2p"
    assert d["lane_is_framework"] is False  # forced by name: RCCL's own collectives
    assert d["groups_per_round"] == 2.0


def test_bench_lane_select():
    """--lane auto at N>1: each of the framework's lanes is checked exact and
    timed before the warmup, and the timed rounds run on the faster one (every
    rank agrees).  RCCL's own collectives are never a candidate: they are the
    comparator (other_lane)."""
    d = _run(3)
    sel = d["lane_select"]
    # the default (pruned) set on CPU processes: the p2p schedule alone
    assert [k for k in sel if k != "chosen"] == ["p2p"], sel
    assert sel["chosen"] == "p2p" and d["lane"] == "p2p"
    assert sel["p2p"]["exact"] is True and sel["p2p"]["ms"] > 0
    assert sel["p2p"]["burst"] == {"rounds": 32, "bad_elements_max_rank": 0}
    assert "collective" not in sel and d["lane_is_framework"] is True
    assert d["other_lane"]["lane"] == "collective"
    assert d["exact"] is True and d["groups_per_round"] > 0


def test_bench_n8_full_flow():
    """The driver's largest N: 8 ranks through preflight, lane selection,
    timed rounds, check, comparator and the other lane (uneven blocks: 0.3 MiB
    of fp32 = 78643 elements over 8 ranks, 16 KiB chunks)."""
    d = _run(8, "--size-mb", "0.3", "--chunk-mb", "0.015625")
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8" and d["exact"] is True
    assert d["p2p_nranks"] == 8 and [r["rank"] for r in d["rank_devices"]] == list(range(8))
    sel = d["lane_select"]
    assert sel["p2p"]["exact"] is True and "collective" not in sel
    assert d["lane"] == sel["chosen"] and d["xgmi_bound_algbw_GBps"] == pytest.approx(612.0, abs=1.0)
    assert abs(d["busbw_GBps"] - d["value"] * 2 * 7 / 8) < 1e-2


def test_bench_multirank_extras_deadline():
    """The extras' deadline ends every rank mid-config: the processes rank 0
    started for config 1 (a master and 2 workers, bench.run_cfg1) must not
    outlive it (the native watchdog kills the children it tracks)."""
    import time

    import psutil

    t0 = time.time()
    d = _run(2, "--extras", "on", "--extras-deadline-s", "0.05")
    assert d["exact"] is True and "extras_error" in d and "extra_configs" not in d
    assert d["value"] > 0
    time.sleep(0.5)
    left = []
    for p in psutil.process_iter(["pid", "ppid", "cmdline", "create_time"]):
        cmd = " ".join(p.info["cmdline"] or [])
        if p.info["ppid"] == 1 and "akka_allreduce_amd" in cmd and p.info["create_time"] >= t0 - 1:
            left.append((p.info["pid"], cmd[:120]))
    assert not left, left


def test_bench_stalled_rank_fails_legibly():
    """A rank that never posts its side of the preflight round: rank 0 must
    print ONE failure line naming the phase inside the preflight deadline and
    the job must exit non-zero (no hang until an outer limit)."""
    import time

    t0 = time.monotonic()
    d = _run(2, "--preflight-deadline-s", "8", env={"AKKA_FAULT_STALL_RANK": "1", "AKKA_FAULT_STALL_PHASE": "preflight"},
             expect_rc=1)
    assert time.monotonic() - t0 < 90
    assert d["failed_phase"] == "preflight" and d["value"] is None
    assert "deadline" in d["failure"] and "rccl_debug_tail" in d
    assert d["phases_passed"] == ["init", "rccl_init", "identity"]


def test_bench_rank_error_reported_by_rank0():
    """A Python error on rank 1 reaches rank 0 through the agreement step."""
    d = _run(2, env={"AKKA_FAULT_STALL_RANK": "1", "AKKA_FAULT_STALL_PHASE": "warmup", "AKKA_FAULT_STALL_MODE": "raise"},
             expect_rc=1)
    assert d["failed_phase"] == "warmup"
    # either through the agreement step or through the failure beacon
    assert "injected fault on rank 1" in json.dumps(d), d


def test_bench_cfg4_threshold_straggler():
    """BASELINE config 4 in the bench extras on the one-sided lane (0.75/0.75,
    maxLag 1, rank N-1 sleeps before each call), 48 rounds per phase -- steady
    state.  At N=4 three of four contributions reduce a chunk and 3/4 of the
    chunks complete a round, so the fast ranks never wait for the straggler:
    their median and p90 per round stay far below its delay, its late pushes
    are dropped, its calls catch up.  (At N=2/3, 0.75 of the chunks always
    includes the straggler's block -- the reference's semantics.)"""
    delay = 100.0
    d = _run(4, "--extras", "on", "--extras-only", "cfg4", "--cfg4-size-mb", "1", "--cfg4-delay-ms", str(delay),
             "--cfg4-rounds", "48")
    c = d["extra_configs"]["cfg4_threshold_straggler"]
    assert c["straggler_rank"] == 3 and c["thresholds"] == [1.0, 0.75, 0.75] and c["max_lag"] == 1
    assert c["transport"] == "onesided" and c["rounds_per_phase"] == 48
    w = c["with_straggler"]
    assert w["fast_rank_median_ms_per_round"] < delay / 10, c
    assert w["fast_rank_p90_ms_per_round"] < delay / 3, c
    assert all(n >= 24 for n in w["fast_rank_calls"]) and w["straggler_calls"] < 48, c
    assert w["catch_up_skipped_rounds"] > 0 and w["timeouts"] == 0, c
    assert 0 < w["fast_rank_mean_count"] <= 3
    assert "fast_rank_slowdown" in c and c["no_straggler"]["timeouts"] == 0
    # at N=4 the three fast blocks alone meet floor(0.75 * 4) = 3 (one chunk per block here)
    assert c["straggler_block_required"] is False and c["need_complete_chunks"] == 3
    assert c["total_chunks"] == 4 and c["straggler_chunks"] == 1 and c["straggler_copy_required"] is False
    # the untimed validation rounds: 2^rank inputs, every chunk's set matches its count
    v = c["validation"]
    assert v["contributor_sets_consistent"] is True and v["bad_chunks"] == 0 and v["chunks_checked"] >= 4 * 12, v
    ck = d["checks"]  # the line's summary of the job's own checks
    assert ck["cfg4_contributor_sets_consistent"] is True and ck["cfg4_chunks_checked"] == v["chunks_checked"], ck


def test_bench_cfg4_n2_labels_the_straggler_block_as_required():
    """At N=2 with 16 MiB (4 chunks of 4 MiB), floor(0.75 * 4) = 3 chunks
    need one of the straggler's 2: the line says so (straggler_block_required),
    so a slow N=2 point reads as the reference's semantics, not as a
    regression."""
    d = _run(2, "--extras", "on", "--extras-only", "cfg4", "--cfg4-size-mb", "16", "--cfg4-delay-ms", "10",
             "--cfg4-rounds", "6")
    c = d["extra_configs"]["cfg4_threshold_straggler"]
    assert c["straggler_block_required"] is True and c["need_complete_chunks"] == 3, c
    assert c["straggler_chunks"] == 2 and c["need_reduce_copies"] == 1


def test_bench_cfg1_readme_demo():
    """BASELINE config 1 in the bench extras: the reference's README demo as
    a master and 2 worker processes over TCP, with the demo's thresholds and
    with exact thresholds + the sink's assertMultiple check."""
    d = _run(2, "--extras", "on", "--extras-only", "cfg1")
    c = d["extra_configs"]["cfg1_readme_demo_cluster"]
    for tag in ("demo_thresholds", "exact_assert"):
        assert c[tag]["rcs"] == [0, 0, 0], c
        assert all(r and r > 0 for r in c[tag]["rounds_per_s"]), c
    assert c["exact_assert"]["failures"] == [0, 0]
