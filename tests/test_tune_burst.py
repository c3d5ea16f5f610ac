"""tune()'s validation burst: a lite candidate whose
output is wrong in ONE element of ONE of its 32 back-to-back burst rounds on
ONE rank is disqualified on every rank, and its fenced twin is chosen; the
result records the burst of every candidate.  CPU processes (gloo), the
one-sided lane over shared memory -- the same lane code and tune() logic as
on the GPU.  The fault is injected into the lane's output in tune()
(AKKA_FAULT_CORRUPT_LANE), standing in for a data-after-flag reorder."""
import json
import os
import subprocess
import sys
import tempfile

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_onesided_cpu import ROOT, _free_port  # noqa: E402


def run(n, *extra, env=None, timeout=300):
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "tune_ranks.py"), "--out-dir", out, *extra]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT,
                           env={**os.environ, **(env or {})})
        assert r.returncode == 0, r.stderr[-3000:]
        return [json.load(open(os.path.join(out, f"rank{i}.json"))) for i in range(n)]


def test_clean_burst_keeps_both_handoffs():
    rows = run(2)
    for d in rows:
        t = d["tune"]
        for c in ("onesided", "onesided_fenced"):
            assert t[c]["exact"] is True and t[c]["burst"] == {"rounds": 32, "bad_elements_max_rank": 0}, t
        assert t["chosen"] in ("onesided", "onesided_fenced")
        assert d["exact_after"] == [True] * 3
    assert len({d["tune"]["chosen"] for d in rows}) == 1  # every rank agrees


@pytest.mark.parametrize("n,bad_rank,dtype", [(2, 1, "float32"), (3, 2, "bfloat16")])
def test_one_corrupt_round_disqualifies_the_lite_lane(n, bad_rank, dtype):
    rows = run(n, "--dtype", dtype, env={"AKKA_FAULT_CORRUPT_LANE": "onesided",
                                         "AKKA_FAULT_CORRUPT_RANK": str(bad_rank),
                                         "AKKA_FAULT_CORRUPT_ROUND": "19"})
    for d in rows:
        t = d["tune"]
        # disqualified on EVERY rank, although only one rank saw the bad element
        assert t["onesided"]["exact"] is False and t["onesided"]["ms"] is None, t
        assert t["onesided"]["burst"]["bad_elements_max_rank"] == 1, t
        assert t["onesided_fenced"]["exact"] is True
        assert t["onesided_fenced"]["burst"]["bad_elements_max_rank"] == 0
        assert t["chosen"] == "onesided_fenced" and d["state_lane"] == "onesided_fenced"
        assert d["exact_after"] == [True] * 3
    assert "burst: 1 wrong elements" in rows[bad_rank]["tune"]["onesided"]["error"]
