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
