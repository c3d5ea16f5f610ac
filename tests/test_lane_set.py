"""First contact with a node: the lanes tune() chooses
among by default, each exact fast lane next to its FENCED twin, and config 4
switching its one-sided lane to the fenced hand-off when its validation
rounds find a bad chunk (the straggler path stays available whatever the
link does, AllreduceWorker.scala:170-186).  CPU only."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from akka_allreduce_amd.parallel import ThresholdAllreduce  # noqa: E402

DEFAULT = ["p2p", "ipc_lite_direct", "ipc_fused_lite_direct", "ipc_fused_direct", "onesided", "onesided_fenced"]


def test_default_candidates_are_pruned_with_fenced_twins():
    c = ThresholdAllreduce.lane_candidates(two_sided=True, ipc_open=True, onesided_ok=True)
    assert c == DEFAULT and len(c) <= 6
    # every candidate is a lane the engine knows; the fast lite lanes each
    # have a fenced twin in the set (lite flag False)
    for name in c:
        assert name in ThresholdAllreduce.LANES
    assert ThresholdAllreduce.LANES["ipc_fused_direct"][5] is False
    assert ThresholdAllreduce.LANES["ipc_fused_lite_direct"][5] is True
    assert ThresholdAllreduce.LANES["onesided_fenced"][0] == "onesided"


def test_lane_table_is_pruned():
    """at most 8 lanes, the comparator included; no
    measurement-only variants (engine-path ipc modes, p2p_block) and no
    'all' candidate set."""
    assert len(ThresholdAllreduce.LANES) <= 8
    assert set(ThresholdAllreduce.LANES) == {"collective", "p2p", "ipc_fused_lite", "ipc_lite_direct",
                                            "ipc_fused_lite_direct", "ipc_fused_direct", "onesided",
                                            "onesided_fenced"}
    with pytest.raises(TypeError):
        ThresholdAllreduce.lane_candidates(two_sided=True, ipc_open=True, onesided_ok=True, lane_set="all")
    # tune() never offers the comparator
    for kw in ({}, {"paced": True}, {"exact": False}):
        assert "collective" not in ThresholdAllreduce.lane_candidates(two_sided=True, ipc_open=True,
                                                                      onesided_ok=True, **kw)


def test_candidates_follow_what_the_job_can_run():
    # ipc-only job (no RCCL communicator): the window lanes alone
    assert ThresholdAllreduce.lane_candidates(two_sided=False, ipc_open=True, onesided_ok=True) == DEFAULT[1:]
    # paced job: no direct rounds (they bypass the pacer); the engine-path
    # fused lite round stands in, p2p is its safe alternative
    c = ThresholdAllreduce.lane_candidates(two_sided=True, ipc_open=True, onesided_ok=True, paced=True)
    assert c == ["p2p", "ipc_fused_lite", "onesided", "onesided_fenced"]
    # windows unavailable: the two-sided lane only
    assert ThresholdAllreduce.lane_candidates(two_sided=True, ipc_open=False, onesided_ok=False) == ["p2p"]


def test_cfg4_switches_to_fenced_handoff_on_bad_validation():
    """AKKA_FAULT_BAD_HANDOFF=lite: rank 1's validation rounds count a torn
    chunk while the lane runs lite hand-offs.  Every rank switches to the
    fenced hand-off, measures both phases again and validates clean; the
    line says so and keeps the lite run."""
    from test_bench_multirank_cpu import _run

    d = _run(4, "--extras", "on", "--extras-only", "cfg4", "--cfg4-size-mb", "1", "--cfg4-delay-ms", "20",
             "--cfg4-rounds", "16", env={"AKKA_FAULT_BAD_HANDOFF": "lite", "AKKA_FAULT_BAD_HANDOFF_RANK": "1"})
    c = d["extra_configs"]["cfg4_threshold_straggler"]
    assert c["handoff"] == "fenced", c
    fb = c["handoff_fallback"]
    assert fb["from"] == "lite" and fb["lite"]["validation"]["contributor_sets_consistent"] is False
    assert fb["lite"]["validation"]["bad_chunks"] > 0 and fb["lite"]["validation"]["handoff"] == "lite"
    v = c["validation"]
    assert v["handoff"] == "fenced" and v["contributor_sets_consistent"] is True and v["bad_chunks"] == 0, v
    for ph in ("no_straggler", "with_straggler"):
        assert ph in c and ph in fb["lite"]
    assert d["checks"]["cfg4_contributor_sets_consistent"] is True


def test_onesided_cpu_fenced_handoff_is_reported_and_exact():
    from test_onesided_cpu import run_ranks

    r, rows = run_ranks(2, "--mode", "exact", "--size", str(1 << 14), "--chunk", str(1 << 11), "--rounds", "3",
                        "--handoff", "fenced")
    assert r.returncode == 0, r.stderr[-3000:]
    for d in rows:
        assert d["info"]["handoff"] == "fenced" and d["exact"] == [True] * 3
