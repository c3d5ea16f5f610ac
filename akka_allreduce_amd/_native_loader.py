"""Loads the in-tree native extension, building it on first use if needed.

The extension is the only implementation of the engine/kernels: there is no
Python fallback, so a missing or broken build fails loudly here.
``AKKA_NATIVE_PATH`` loads an alternative build of the same module (e.g. the
AddressSanitizer variant from ``_build.build(sanitize=...)``).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        import torch  # noqa: F401  (loads torch's HIP runtime + RCCL first: one copy per process)

        alt = os.environ.get("AKKA_NATIVE_PATH")
        if alt:
            spec = importlib.util.spec_from_file_location("akka_allreduce_amd._native", alt)
            mod = importlib.util.module_from_spec(spec)
            sys.modules["akka_allreduce_amd._native"] = mod
            spec.loader.exec_module(mod)
            _mod = mod
            return _mod

        from . import _build

        # A module built from other sources than the ones in the tree (edited
        # kernels, an old .so next to new code) is rebuilt before it is
        # imported -- never silently run; with no compiler here it is an error.
        why = "AKKA_REBUILD=1" if os.environ.get("AKKA_REBUILD") == "1" else _build.stale_reason()
        if why is not None:
            if not _build.have_compiler():
                raise RuntimeError(f"akka_allreduce_amd: the native extension at {_build.ext_path()} must be rebuilt "
                                   f"({why}) but hipcc / g++ are not available here")
            _build.build()
        _mod = importlib.import_module("akka_allreduce_amd._native")
        return _mod
