"""bench.py's driver contract on one MI355X: one JSON line with the metric
and config BASELINE.json names, exact result, timing fields consistent."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_prints_one_baseline_line():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        baseline = json.load(f)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--size-mb", "16", "--extras", "on"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["metric"] == baseline["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2
    assert d["unit"] == "GB/s" and d["higher_is_better"] is True and d["dtype"] == "fp32"
    assert d["exact"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value is the buffer's bytes per second of one round
    assert abs(d["value"] - d["config"]["buffer_bytes"] / (d["ms_per_step"] * 1e-3) / 1e9) / d["value"] < 0.05  # ms_per_step is rounded to 0.1 us
    ex = d["extra_configs"]
    assert ex["cfg3_bf16_1GiB_chunk8MiB"]["algbw_GBps"] > 0, ex
    assert ex["cfg5_mlp_dp_sgd"]["steps_per_s"] > 0, ex
    assert ex["cfg5_mlp_dp_sgd_bf16_graph"]["steps_per_s"] > 0, ex


def test_bench_extras_deadline_keeps_headline():
    """Extras that overrun their deadline are dropped; the headline line still prints once, rc 0."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--size-mb", "16", "--extras", "on", "--extras-deadline-s", "0.01"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["exact"] is True and d["value"] > 0
    assert "extras_error" in d and "extra_configs" not in d


@pytest.mark.parametrize("plane", ["ipc", "ipc_p2p"])
def test_bench_multirank_on_one_card(plane):
    """The driver's N>1 invocation (torch.distributed.run, one process per
    rank) on the box's one GPU: ranks share the card (AKKA_SHARE_GPU=1) with a
    data plane that needs no RCCL communicator.  One line, every phase passed,
    every lane candidate exact, the chosen lane timed, cfg4 from the fast ranks'
    side.  (Numbers are HBM-local, not the metric.)"""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n = 4 if plane == "ipc_p2p" else 2
    extra = ["--extras", "on", "--extras-only", "cfg4", "--cfg4-size-mb", "4", "--cfg4-delay-ms", "40",
             "--cfg4-rounds", "48"] if plane == "ipc_p2p" else ["--extras", "off"]
    env = dict(os.environ, AKKA_SHARE_GPU="1", GPU_MAX_HW_QUEUES="8")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(n), "--steps", "4", "--warmup", "2", "--size-mb", "16", "--data-plane", plane,
                        "--compare-rccl", "off", *extra],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["exact"] is True and d["preflight"] == "passed" and d["value"] > 0
    assert d["config"]["data_plane"] == plane and d["p2p_nranks"] == n
    sel = d["lane_select"]
    cands = [k for k in sel if k != "chosen"]
    assert all(sel[k]["exact"] is True for k in cands), sel
    # every candidate passed tune()'s validation burst (32 back-to-back rounds)
    assert all(sel[k]["burst"] == {"rounds": 32, "bad_elements_max_rank": 0} for k in cands), sel
    assert d["lane"] == sel["chosen"]
    lp = d["link_probe"]  # the N x N matrix, labelled: ranks share one card, not xGMI
    assert "share ONE GPU" in lp["note"] and len(lp["push_GBps"]) == n and len(lp["pull_GBps"][0]) == n
    assert all(lp["push_GBps"][i][j] > 0 for i in range(n) for j in range(n) if i != j)
    if plane == "ipc_p2p":
        # the default (pruned) lane set: the p2p schedule, the direct ipc
        # rounds with the fused round's fenced twin, the one-sided lane in
        # both hand-off modes (<= 6 candidates at first contact)
        assert cands == ["p2p", "ipc_lite_direct", "ipc_fused_lite_direct", "ipc_fused_direct", "onesided",
                         "onesided_fenced"], cands
        assert d["lane_is_framework"] is True
        c4 = d["extra_configs"]["cfg4_threshold_straggler"]
        w = c4["with_straggler"]
        assert c4["transport"] == "onesided" and w["timeouts"] == 0, c4
        assert w["fast_rank_median_ms_per_round"] < 40 / 4 and w["catch_up_skipped_rounds"] > 0, c4
        # the untimed validation rounds (2^rank inputs): every chunk's set matches its count
        v = c4["validation"]
        assert v["contributor_sets_consistent"] is True and v["bad_chunks"] == 0, v
        assert c4["handoff"] == "lite" and c4["handoff_fallback"] is None, c4
    else:
        # ipc-only job: the window lanes of the default set
        assert cands == ["ipc_lite_direct", "ipc_fused_lite_direct", "ipc_fused_direct", "onesided",
                         "onesided_fenced"], cands


def test_bench_rccl_init_failure_falls_back_to_ipc():
    """RCCL init raising on EVERY rank (injected: AKKA_FAULT_STALL_RANK=all,
    phase rccl_init, mode raise) does not cost the headline: the job is rebuilt
    in the same processes on the ipc data plane and the line says so."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, AKKA_SHARE_GPU="1", GPU_MAX_HW_QUEUES="8", AKKA_FAULT_STALL_RANK="all",
               AKKA_FAULT_STALL_PHASE="rccl_init", AKKA_FAULT_STALL_MODE="raise")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--size-mb", "16", "--compare-rccl", "off",
                        "--extras", "off"], capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["rccl_fallback"]["data_plane"] == "ipc" and set(d["rccl_fallback"]["rccl_init_errors"]) == {"0", "1"}
    assert d["config"]["data_plane"] == "ipc" and (d["lane"].startswith("ipc") or d["lane"].startswith("onesided")) \
        and d["lane_is_framework"] is True
    assert d["exact"] is True and d["value"] > 0


def test_bench_preflight_failure_falls_back_to_ipc():
    """The two-sided default lane failing its preflight on EVERY rank
    (injected: phase preflight, mode raise; the mailbox p2p data plane stands
    in for RCCL on a shared card) does not cost the headline: the job checks
    and times the one-sided ipc lanes only, and the line says so."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, AKKA_SHARE_GPU="1", GPU_MAX_HW_QUEUES="8", AKKA_FAULT_STALL_RANK="all",
               AKKA_FAULT_STALL_PHASE="preflight", AKKA_FAULT_STALL_MODE="raise")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--size-mb", "16", "--data-plane", "ipc_p2p",
                        "--extras", "off", "--link-probe", "off"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert set(d["preflight_fallback"]["errors"]) == {"0", "1"}, d
    assert d["preflight"] == "passed on the ipc lane"
    assert (d["lane"].startswith("ipc") or d["lane"].startswith("onesided")) \
        and d["lane_is_framework"] is True
    assert all(k.startswith("ipc") or k.startswith("onesided") for k in d["lane_select"] if k != "chosen"), \
        d["lane_select"]
    assert d["exact"] is True and d["value"] > 0 and d["rccl_allreduce_algbw_GBps"] is None


def test_bench_cfg5_two_ranks_on_one_card():
    """BASELINE config 5 (MLP DP-SGD) in bench.py's N-rank flow, 2 processes
    on the card, ipc data plane: the eager, graphed and -- on a window lane --
    whole-step graphed variants all run (a one-sided round waiting on its
    peer must not hold the peer's GEMMs off the card: cu_keep on a shared
    GPU, profiles/r04/README.md)."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, AKKA_SHARE_GPU="1", GPU_MAX_HW_QUEUES="8")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--size-mb", "16", "--data-plane", "ipc",
                        "--extras", "on", "--extras-only", "cfg5", "--link-probe", "off", "--compare-rccl", "off",
                        "--extras-deadline-s", "150"], capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    d = json.loads(lines[-1])
    assert "extras_error" not in d, d.get("extras_error")
    ex = d["extra_configs"]
    assert "cfg5_error" not in ex, ex.get("cfg5_error")
    for k in ("cfg5_mlp_dp_sgd", "cfg5_mlp_dp_sgd_bf16", "cfg5_mlp_dp_sgd_bf16_graph"):
        assert ex[k]["steps_per_s"] > 50, ex
    if d["lane"].startswith("onesided") or d["lane"].startswith("ipc"):
        w = ex["cfg5_mlp_dp_sgd_bf16_whole_graph"]
        assert w["lane"] == d["lane"] and w["steps_per_s"] > 50, ex
