"""The native phase watchdog (csrc/runtime/watchdog.cpp): fires without the
GIL, writes the pre-composed line with the reason and the debug-log tail
spliced in, exits with the given code; disarm cancels; a failure beacon
written by another rank fires it early; SIGTERM writes the line too."""
import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(body: str, timeout=60):
    code = ("import sys, time; sys.path.insert(0, %r)\n"
            "from akka_allreduce_amd._native_loader import load\n"
            "n = load()\n" % ROOT) + body
    return subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def test_json_escape(native):
    assert native.json_escape('a"b\\c\nd\te\x01') == 'a\\"b\\\\c\\nd\\te\\u0001'


def test_fires_with_reason_and_tail(tmp_path):
    log = tmp_path / "rccl.log"
    log.write_text("line one\nNCCL WARN peer 3 unreachable\n")
    line = json.dumps({"failed_phase": "preflight", "failure": "__AKKA_REASON__", "tail": "__AKKA_TAIL__"})
    p = _child(f"n.watchdog_arm(0.5, {line!r}, True, {str(log)!r}, 7, 4096)\n"
               "time.sleep(30)  # holds the GIL in a sleep loop; the native thread still fires\n")
    out, err = p.communicate(timeout=60)
    assert p.returncode == 7
    d = json.loads(out.strip().splitlines()[-1])
    assert d["failed_phase"] == "preflight" and "deadline" in d["failure"]
    assert "peer 3 unreachable" in d["tail"]


def test_disarm_cancels():
    p = _child("n.watchdog_arm(0.3, '{\"x\": 1}', True, '', 9, 64)\nn.watchdog_disarm()\ntime.sleep(1.0)\n"
               "print('survived')\n")
    out, _ = p.communicate(timeout=60)
    assert p.returncode == 0 and "survived" in out


def test_beacon_fires_early(tmp_path):
    beacon = tmp_path / "beacon"
    p = _child(f"n.watchdog_arm(60, '{{\"why\": \"__AKKA_REASON__\"}}', True, '', 5, 64, {str(beacon)!r})\n"
               "time.sleep(60)\n")
    time.sleep(1.0)
    beacon.write_text("rank 2 failed in warmup: boom")
    t0 = time.monotonic()
    out, _ = p.communicate(timeout=60)
    assert time.monotonic() - t0 < 10
    assert p.returncode == 5
    assert "rank 2 failed in warmup" in json.loads(out.strip().splitlines()[-1])["why"]


def test_sigterm_writes_the_line():
    p = _child("n.watchdog_install_sigterm()\nn.watchdog_arm(60, '{\"why\": \"__AKKA_REASON__\"}', True, '', 4, 64)\n"
               "print('armed', flush=True)\ntime.sleep(60)\n")
    assert p.stdout.readline().strip() == "armed"
    p.send_signal(signal.SIGTERM)
    out, _ = p.communicate(timeout=60)
    assert p.returncode == 4
    assert json.loads(out.strip().splitlines()[-1])["why"] == "SIGTERM"


def test_fire_kills_tracked_children():
    """A watchdog exit skips Python's `finally` blocks: the children a rank
    registered (bench.py config 1's master and workers) are killed with it,
    untracked ones are not."""
    p = _child("import subprocess\n"
               "def sl(): return subprocess.Popen(['sleep', '120'], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)\n"
               "a = sl(); b = sl(); c = sl()\n"
               "assert n.watchdog_track_child(a.pid) and n.watchdog_track_child(b.pid) and n.watchdog_track_child(c.pid)\n"
               "n.watchdog_untrack_child(c.pid)\n"
               "print(a.pid, b.pid, c.pid, flush=True)\n"
               "n.watchdog_arm(0.5, '{}', True, '', 6, 64)\n"
               "time.sleep(30)\n")
    out, _ = p.communicate(timeout=60)
    assert p.returncode == 6
    a, b, c = (int(v) for v in out.split()[:3])
    time.sleep(0.3)

    def alive(pid):
        try:  # (an orphan killed by SIGKILL is reaped by init: gone, or a zombie)
            with open(f"/proc/{pid}/stat") as f:
                return f.read().split(")")[-1].split()[0] != "Z"
        except FileNotFoundError:
            return False

    assert not alive(a) and not alive(b)
    assert alive(c)
    os.kill(c, signal.SIGKILL)
