"""roctx ranges/markers (visible in rocprofv3 --marker-trace timelines).

The reference has no tracing beyond ``log.debug`` per message.
Here a round and its phases can be bracketed with roctx ranges.  Enabled with
``AKKA_TRACE=1`` (otherwise every call is a no-op costing one attribute load).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterator, Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("AKKA_TRACE", "0") == "1"


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _enabled
    if _lib is not None or not _enabled:
        return _lib
    cands = []
    try:
        import torch

        cands.append(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:  # pragma: no cover
        pass
    cands += ["/opt/rocm/lib/libroctx64.so", "libroctx64.so"]
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            return _lib
        except OSError:
            continue
    _enabled = False
    return None


def enabled() -> bool:
    return _enabled and _load() is not None


def set_enabled(flag: bool) -> None:
    global _enabled
    _enabled = bool(flag)


def mark(msg: str) -> None:
    if _enabled and _load():
        _lib.roctxMarkA(msg.encode())


@contextlib.contextmanager
def range_(msg: str) -> Iterator[None]:
    if not (_enabled and _load()):
        yield
        return
    _lib.roctxRangePushA(msg.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()
