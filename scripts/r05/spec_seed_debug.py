"""Replay test_random_orders_match_reference_rules(seed) on the GPU window
harness with a log line per step (time, injected message, outputs, stats)."""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_onesided_spec as spec  # noqa: E402
import test_onesided_spec_gpu as sg  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
orig_scatter, orig_reduce = sg.WindowSpecHarness.scatter, sg.WindowSpecHarness.reduce
t0 = time.monotonic()


def log(h, what):
    st = h.stats()
    print(f"{time.monotonic() - t0:7.3f}s {what}: outputs={[(o[0], o[3]) for o in h.outputs]} "
          f"sent={len(h.sent)} w={ {k: v for k, v in st.items() if v} }", flush=True)


def scatter(self, src, k, r, vals):
    orig_scatter(self, src, k, r, vals)
    log(self, f"scatter s{src} k{k} r{r} {vals} peer-stats={ {a: b for a, b in self.stats(src).items() if b} }")


def reduce(self, src, k, r, count, vals):
    orig_reduce(self, src, k, r, count, vals)
    log(self, f"reduce s{src} k{k} r{r} c{count} {vals} peer-stats={ {a: b for a, b in self.stats(src).items() if b} }")


orig_start, orig_settle = sg.WindowSpecHarness.start, sg.WindowSpecHarness.settle


def start(self, data):
    print(f"{time.monotonic() - t0:7.3f}s start {data}", flush=True)
    orig_start(self, data)
    log(self, "started")


def settle(self):
    ts = time.monotonic()
    orig_settle(self)
    print(f"{time.monotonic() - t0:7.3f}s   settle took {time.monotonic() - ts:.3f}s sig={self._sig()}", flush=True)


sg.WindowSpecHarness.start = start
sg.WindowSpecHarness.settle = settle
sg.WindowSpecHarness.scatter = scatter
sg.WindowSpecHarness.reduce = reduce
if len(sys.argv) > 2 and sys.argv[2] == "cpu":
    H = sg.CpuWindowSpecHarness
else:
    H = sg.WindowSpecHarness
spec.SpecHarness = H
try:
    spec.test_random_orders_match_reference_rules(seed)
    print("PASS")
except AssertionError as e:
    import traceback
    traceback.print_exc()
    print("FAIL", e)
finally:
    while sg._OPEN:
        sg._OPEN.pop().close()
