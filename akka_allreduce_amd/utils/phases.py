"""Phase guard for multi-rank jobs: every phase has a deadline, every rank
agrees on its outcome, and a failure ends the job with ONE legible line.

A job that loses a peer (RCCL init never completes, a p2p group never
matches, a rank crashed) must not sit until an outer time limit kills it
without a trace.  ``PhaseGuard`` gives each phase:

* a native watchdog (``csrc/runtime/watchdog.cpp``): a C++ thread that needs
  neither the GIL nor HIP, so it still fires while the main thread is stuck
  inside ``ncclCommInitRank`` / ``ncclGroupEnd`` / a stream synchronize.  On
  expiry (or SIGTERM from the launcher) it writes the failure line, with the
  tail of this rank's RCCL debug log, and exits non-zero;
* an agreement step: each rank's outcome (``None`` or the error text) is
  all-gathered over the host process group, so a Python error on one rank is
  reported by rank 0 for everyone instead of turning into a hang elsewhere;
* a faulthandler stack dump shortly before the watchdog fires.

The reference's only liveness mechanism is the Akka failure detector
(``auto-down-unreachable-after = 10s``, application.conf:18-20) plus master
DeathWatch (AllreduceMaster.scala:46-52); it has no notion of a failed phase.
"""
from __future__ import annotations

import faulthandler
import json
import os
import sys
from typing import Any, Callable, Dict, List, Optional

REASON = "__AKKA_REASON__"
TAIL = "__AKKA_TAIL__"


def rccl_debug_path(rank: int) -> str:
    """Per-rank RCCL debug log: set NCCL_DEBUG=WARN + NCCL_DEBUG_FILE before
    the first RCCL call (unless the user chose their own)."""
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"akka_rccl_debug.r{rank}.{os.getpid()}.log")


def default_beacon_path() -> str:
    """Failure beacon shared by the ranks of one launcher invocation (all
    ranks of a node are children of the same torchrun process)."""
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"akka_fail_beacon.{os.getppid()}.{port}")


def enable_rccl_debug_log(rank: int) -> str:
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    return os.environ.setdefault("NCCL_DEBUG_FILE", rccl_debug_path(rank))



def progress(msg: str) -> None:
    """One timestamped line on stderr (bench.py's stdout is reserved for the
    JSON result): a long multi-rank run shows where each rank is."""
    import sys
    import time

    print(f"[akka {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)

class PhaseGuard:
    def __init__(self, base: Dict[str, Any], rank: int, world: int, debug_path: str = "",
                 exit_code: int = 3, stream=None, beacon_path: Optional[str] = None):
        from .._native_loader import load

        self._n = load()
        self.base = dict(base)
        self.rank = rank
        self.world = world
        self.debug_path = debug_path
        self.exit_code = exit_code
        self.phase: Optional[str] = None
        self.history: List[str] = []
        self.stream = stream or sys.stdout
        self.beacon_path = (default_beacon_path() if world > 1 else "") if beacon_path is None else beacon_path
        self._n.watchdog_install_sigterm()

    # ------------------------------------------------------------------ lines
    def failure_line(self, phase: str, failure: str, errors: Optional[Dict[int, str]] = None,
                     tail: Optional[str] = None) -> Dict[str, Any]:
        d = dict(self.base)
        d["value"] = None
        d["failed_phase"] = phase
        d["failure"] = failure
        d["phases_passed"] = list(self.history)
        d["reporting_rank"] = self.rank
        if errors:
            d["rank_errors"] = {str(k): v for k, v in errors.items()}
        d["rccl_debug_tail"] = tail if tail is not None else TAIL
        return d

    def arm(self, seconds: float, line: Optional[Dict[str, Any]], exit_code: Optional[int] = None,
            watch_beacon: bool = True) -> None:
        """Low-level: arm the native watchdog with an arbitrary line (rank 0
        writes it to stdout, other ranks to stderr)."""
        text = json.dumps(line) if line is not None else ""
        self._n.watchdog_arm(float(seconds), text, self.rank == 0, self.debug_path,
                             self.exit_code if exit_code is None else int(exit_code), 4096,
                             self.beacon_path if watch_beacon else "")
        # Python stacks of every thread go to stderr just before the native exit.
        faulthandler.dump_traceback_later(max(0.5, float(seconds) - 1.0), exit=False)

    def disarm(self) -> None:
        self._n.watchdog_disarm()
        faulthandler.cancel_dump_traceback_later()

    # ------------------------------------------------------------------ phases
    def enter(self, phase: str, seconds: float) -> None:
        self.phase = phase
        self.arm(seconds, self.failure_line(phase, REASON))

    def run(self, phase: str, seconds: float, fn: Callable[[], Any], agree: bool = True) -> Any:
        """Run ``fn`` as ``phase`` under a deadline; with ``agree`` every rank
        learns every other rank's outcome before the next phase starts."""
        self.enter(phase, seconds)
        err = None
        result = None
        progress(f"rank {self.rank}: phase {phase} (deadline {seconds:g} s)")
        try:
            result = fn()
        except Exception as e:  # reported through the agreement step (or directly)
            err = f"{type(e).__name__}: {e}"[:600]
            # peers may be stuck waiting for this rank (and never reach the
            # agreement): raise the beacon so their watchdogs fire now, and
            # make sure this rank's own line carries its error
            self.raise_beacon(phase, err)
            self.arm(min(float(seconds), 60.0), self.failure_line(phase, REASON, {self.rank: err}),
                     watch_beacon=False)
        if agree and self.world > 1:
            errors = self._gather(phase, err)
        else:
            errors = {self.rank: err} if err else {}
        if errors:
            self.fail(phase, "error", errors)
        self.disarm()
        self.history.append(phase)
        self.phase = None
        return result

    def try_run(self, phase: str, seconds: float, fn: Callable[[], Any]) -> tuple:
        """Like ``run``, but an error that every rank AGREES on is returned
        (result, {rank: error}) instead of ending the job, so the caller can
        fall back (bench.py: RCCL init failing everywhere -> the ipc lane).  A
        hang still ends the job at the deadline; no beacon is raised, so ranks
        that fail a little later still reach the agreement."""
        self.enter(phase, seconds)
        err = None
        result = None
        progress(f"rank {self.rank}: phase {phase} (deadline {seconds:g} s, fallback allowed)")
        try:
            result = fn()
        except Exception as e:
            err = f"{type(e).__name__}: {e}"[:600]
        errors = self._gather(phase, err) if self.world > 1 else ({self.rank: err} if err else {})
        self.disarm()
        self.history.append(phase if not errors else f"{phase}:failed")
        self.phase = None
        return result, errors

    def raise_beacon(self, phase: str, err: str) -> None:
        if not self.beacon_path:
            return
        tmp = f"{self.beacon_path}.{os.getpid()}.tmp"
        try:
            with open(tmp, "w") as f:
                f.write(f"rank {self.rank} failed in {phase}: {err}"[:1500])
            os.replace(tmp, self.beacon_path)  # atomic: readers never see half a message
        except OSError:
            pass

    def _gather(self, phase: str, err: Optional[str]) -> Dict[int, str]:
        import torch.distributed as dist

        obj: List[Any] = [None] * self.world
        try:
            dist.all_gather_object(obj, err)
        except Exception as e:  # a peer died: its socket closed under the gather
            return {self.rank: err or f"agreement after {phase} failed: {type(e).__name__}: {e}"[:600]}
        return {i: o for i, o in enumerate(obj) if o}

    def fail(self, phase: str, failure: str, errors: Optional[Dict[int, str]] = None) -> None:
        """Write the failure line (rank 0: stdout) and exit non-zero now."""
        self.disarm()
        tail = ""
        if self.debug_path and os.path.exists(self.debug_path):
            with open(self.debug_path, "rb") as f:
                f.seek(0, os.SEEK_END)
                n = f.tell()
                f.seek(max(0, n - 4096))
                tail = f.read().decode("utf-8", "replace")
        line = json.dumps(self.failure_line(phase, failure, errors, tail))
        out = self.stream if self.rank == 0 else sys.stderr
        print(line, file=out, flush=True)
        if self.rank != 0:
            print(f"rank {self.rank}: phase {phase} failed: {errors}", file=sys.stderr, flush=True)
        sys.stderr.flush()
        os._exit(self.exit_code + 1)
