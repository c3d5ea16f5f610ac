"""The one-sided xGMI lane (csrc/transport/ipc_lane.h, csrc/kernels/ipc.hip)
with real processes: 2-3 ranks share the one GPU of the box, each maps the
others' windows through IPC handles, and every round is checked bitwise
against the fp32 sum in ascending source order (the kernel's order) on the
CPU.  Covers even/uneven geometries (vector and scalar paths), bf16, empty
blocks, and a missing peer: the bounded waits turn it into ipc_error != 0 on
the others instead of a hung GPU."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, *extra, env=None, timeout=180):
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "ipc_ranks.py"), "--out-dir", out, *extra]
        e = dict(os.environ)
        e.update(env or {})
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=e)
        rows = []
        for i in range(n):
            path = os.path.join(out, f"rank{i}.json")
            if os.path.exists(path):
                with open(path) as f:
                    rows.append(json.load(f))
    return r, rows


@pytest.mark.parametrize("n,size,dtype", [
    (2, 1 << 20, "float32"),      # even blocks: 16-B vector paths
    (3, 1 << 20, "float32"),      # 3 blocks of 349526/349525/349525: scalar paths
    (2, 3 * (1 << 18) + 8, "bfloat16"),
    (3, 2, "float32"),            # S < N: an empty block
    (2, 5 << 20, "float32"),      # several portions per block
    (4, 1 << 24, "float32"),      # 64 MiB: more waiting workgroups than the grid cap (ranks share the card)
])
def test_ipc_lane_exact(n, size, dtype):
    r, rows = _run(n, "--size", str(size), "--dtype", dtype, "--rounds", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(rows) == n
    for d in rows:
        assert d["lane"] == "ipc" and d["ipc_error"] == 0, d
        assert d["exact"] == [True] * 4, d
        assert d["ipc_rounds"] == 4 and d["ipc"]["rounds"] == 4
        assert d["ipc"]["ranks_on_this_gpu"] == n and d["ipc"]["max_wgs"] == max(64, 1024 // n)


@pytest.mark.parametrize("n,size,mode", [
    (2, 1 << 20, "bcast"),
    (3, 1 << 20, "bcast"),        # scalar paths
    (3, 5 << 20, "alternate"),    # pull / bcast every other round: round-id flags serve both
    (4, 1 << 24, "bcast"),
    (3, 5 << 20, "fused"),        # one launch per round, roles pipelined by portion
    (4, 1 << 24, "fused_bcast"),
    (2, 786440, "rotate"),        # pull / bcast / fused pull / fused bcast, round by round (scalar paths)
])
def test_ipc_lane_bcast_mode(n, size, mode):
    """Phase 2 as remote writes (each reducer stores its rows into every
    peer's gather slot, a local copy moves them into the output), and the
    fused single-launch round, in either phase-2 mode."""
    r, rows = _run(n, "--size", str(size), "--rounds", "4", "--mode", mode)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(rows) == n
    for d in rows:
        assert d["ipc_error"] == 0 and d["exact"] == [True] * 4, d
        want_bcast = {"bcast": 4, "fused_bcast": 4, "fused": 0, "alternate": 2, "rotate": 2}[mode]
        assert d["ipc"]["bcast_rounds"] == want_bcast


def test_ipc_lane_missing_peer_times_out_cleanly():
    """Rank 1 leaves after round 0: rank 0's round 1 waits (bounded, 0.5 s)
    for rank 1's flags, reports ipc_error, its next round raises, and the job
    still ends."""
    r, rows = _run(2, "--size", str(1 << 16), "--rounds", "2", "--skip-rank", "1",
                   env={"AKKA_IPC_TIMEOUT_MS": "500"})
    assert r.returncode == 0, r.stderr[-3000:]
    d0 = rows[0]
    assert d0["exact"][0] is True and d0["ipc_error"] != 0, d0
    assert d0["next_round_raised"] is True, d0  # the error surfaces as an exception at the next round
    assert rows[1]["exact"] == [True]


def test_ipc_lane_late_rank_poisons_the_round_everywhere():
    """Rank 1 arrives at round 1 only after rank 0's waits timed out (0.5 s),
    e.g. a rank busy with a checkpoint.  Rank 0 aborts the lane for everyone
    (abort word in every rank's flag area, stored before any of its flags),
    so rank 1 does not consume rank 0's never-written reduced rows either:
    on BOTH ranks round 1's counts are all 0 (never handed back as exact),
    ipc_error is set, and the next round raises."""
    r, rows = _run(2, "--size", str(1 << 16), "--rounds", "2", "--late-rank", "1", "--late-s", "2.0",
                   env={"AKKA_IPC_TIMEOUT_MS": "500"})
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["exact"][0] is True and d["counts_all_zero"] == [False, True], d
        assert d["exact"][1] is False and d["ipc_error"] != 0, d
        assert d["next_round_raised"] is True, d


def test_ipc_round_waits_for_callers_pending_work_on_its_buffers():
    """The round's output and counts are carved from a block that a pending
    kernel on the caller's stream still writes (the caching allocator reuses
    freed memory in that stream's order).  The ipc lane's streams must write
    them only after that point: counts read N, the sum is exact."""
    r, rows = _run(2, "--size", str(1 << 16), "--rounds", "2", "--poison")
    assert r.returncode == 0 and len(rows) == 2, r.stderr[-3000:]
    for d in rows:
        assert d["poison_in_block"], d  # the hazard was really set up
        assert d["poison_counts_ok"] and all(d["exact"]) and d["ipc_error"] == 0, d


def test_ipc_window_too_large_for_one_mapping_fails_fast():
    """A window part of 2 GiB or more (allocations that size hang in
    hipIpcOpenMemHandle, whatever the memory kind: profiles/r03/ipc_open/) is
    refused at construction on every rank, with a message, instead of
    hanging."""
    # N=2 fp32: slot = S/2 elements; the reduced + gather part is 3 slots = 2160 MiB
    r, rows = _run(2, "--size", str(360_000_000), "--rounds", "1", timeout=150)
    assert r.returncode != 0 and not rows
    assert "exceeds the 2047 MiB an IPC mapping opens" in r.stderr, r.stderr[-2000:]


def test_ipc_config3_window_opens_fast():
    """BASELINE config 3's buffer (1 GiB bf16) at N=2: 1.5 GiB window parts,
    below the 2 GiB boundary, map in well under a second and the round is
    exact."""
    r, rows = _run(2, "--size", str(1 << 29), "--dtype", "bfloat16", "--rounds", "1", timeout=200)
    assert r.returncode == 0 and len(rows) == 2, r.stderr[-3000:]
    for d in rows:
        assert d["exact"] == [True] and d["ipc_error"] == 0, d
        assert d["ipc_open_s"] is not None and d["ipc_open_s"] < 1.0, d


@pytest.mark.parametrize("n,size,dtype,mode", [
    (2, 1 << 20, "float32", "rotate"),       # even blocks, all four variants round by round
    (3, 1 << 20, "float32", "alternate"),    # uneven blocks: scalar paths keep their fences
    (2, 3 * (1 << 18) + 8, "bfloat16", "rotate"),
    (4, 1 << 24, "float32", "rotate"),       # many portions
    (8, 1 << 22, "float32", "rotate"),       # a node's rank count: the N=8 reduce kernels
    (8, 1 << 22, "bfloat16", "rotate"),
])
def test_ipc_lane_lite_handoffs(n, size, dtype, mode):
    """AKKA_IPC_LITE=1: fence-free hand-offs (write-through window stores,
    drained flags, system-coherent loads) give the same bitwise sums, across
    XCDs of the card, in every phase-2 mode."""
    r, rows = _run(n, "--size", str(size), "--dtype", dtype, "--mode", mode, "--rounds", "4",
                   env={"AKKA_IPC_LITE": "1", "AKKA_IPC_THREADS": "1024"})
    assert r.returncode == 0 and len(rows) == n, r.stderr[-3000:]
    for d in rows:
        assert all(d["exact"]) and d["ipc_error"] == 0 and d["ipc"]["lite"] is True, d


@pytest.mark.parametrize("threads", [512, 1024])
@pytest.mark.parametrize("n,size,dtype,mode", [
    (2, 1 << 20, "float32", "rotate"),       # even blocks, all four variants round by round
    (3, 1 << 20, "float32", "alternate"),    # uneven blocks: scalar paths, pull / bcast
    (2, 3 * (1 << 18) + 8, "bfloat16", "pull"),
    (4, 1 << 24, "float32", "rotate"),       # many portions, grid cap in waves
])
def test_ipc_lane_wide_workgroups(threads, n, size, dtype, mode):
    """AKKA_IPC_THREADS / set_ipc_mode(threads=...): the round kernels with
    512- or 1024-thread workgroups give the same bitwise sums."""
    r, rows = _run(n, "--size", str(size), "--dtype", dtype, "--mode", mode, "--rounds", "4",
                   env={"AKKA_IPC_THREADS": str(threads)})
    assert r.returncode == 0 and len(rows) == n, r.stderr[-3000:]
    for d in rows:
        assert all(d["exact"]) and d["ipc_error"] == 0, d


def test_ipc_direct_lanes_switch_with_engine_lanes():
    """Direct ipc rounds (device-resident round id, launched on the caller's
    stream) alternating with the engine path and with the fenced direct
    twin: every round exact on every rank, and the lane's round id -- handed
    between host and device at every switch -- advances by one per round."""
    seq = "ipc_lite_direct,ipc_lite_direct,ipc_fused_lite,ipc_fused_direct,ipc_fused_lite_direct,ipc_fused_lite,ipc_lite_direct"
    r, rows = _run(4, "--size", str(1 << 20), "--rounds", "7", "--lane-seq", seq)
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["exact"] == [True] * 7, d
        assert d["counts_all_zero"] == [False] * 7, d
        lr = d["lane_round"]
        assert lr == list(range(lr[0], lr[0] + 7)), lr
    assert len({tuple(d["lane_round"]) for d in rows}) == 1


def test_ipc_direct_lane_missing_peer_raises():
    """Rank 1 leaves after round 0 of a direct ipc lane: rank 0's round 1
    waits (bounded, 0.5 s), its counts table reads 0 (zeroed by the kernel
    whose wait failed, not a fixed N), and its next call raises."""
    r, rows = _run(2, "--size", str(1 << 16), "--rounds", "2", "--skip-rank", "1",
                   "--lane-seq", "ipc_fused_lite_direct", env={"AKKA_IPC_TIMEOUT_MS": "500"})
    assert r.returncode == 0, r.stderr[-3000:]
    d0 = rows[0]
    assert d0["exact"] == [True, False] and d0["ipc_error"] != 0, d0
    assert d0["counts_all_zero"] == [False, True], d0
    assert d0["next_round_raised"] is True, d0
