"""Grouped p2p over ``torch.distributed`` (gloo) for CPU processes.

The native StreamLink issues the same step groups it issues to RCCL on
MI355X; here each group becomes a set of ``isend``/``irecv`` on raw views of
the worker's host buffers, waited together (group semantics).  gloo matches
point-to-point messages per (peer, tag) in issue order -- the same
per-pair FIFO contract as RCCL -- so the production schedule runs unchanged
across real processes on a CPU-only machine (multi-process tests, dev boxes).

``make_async_fns`` is the non-blocking variant used by the reactive transport:
``post(ops)`` starts the sends/receives of one pair group and returns the
pending works, ``test(handle)`` says whether all of them finished.
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Tuple

import torch
import torch.distributed as dist

Op = Tuple[bool, int, int, int, int]  # (send, peer, ptr, nbytes, channel) -- channel = gloo tag


def _view(ptr: int, nbytes: int) -> torch.Tensor:
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return torch.frombuffer(buf, dtype=torch.uint8)


def make_group_fn(group=None) -> Callable[[List[Op]], None]:
    def run(ops: List[Op]) -> None:
        reqs = []
        for send, peer, ptr, nbytes, *ch in ops:
            if nbytes == 0:
                continue
            t = _view(ptr, nbytes)
            tag = ch[0] if ch else 0
            reqs.append(dist.isend(t, peer, group=group, tag=tag) if send else dist.irecv(t, peer, group=group, tag=tag))
        for r in reqs:
            r.wait()

    return run


def make_async_fns(group=None) -> Tuple[Callable[[List[Op]], object], Callable[[object], bool]]:
    """(post, test) for the reactive transport.  gloo's send/recv works only
    complete inside ``wait()``, so each posted group gets a waiter thread
    (``wait`` releases the GIL); ``test`` reads its flag.  Groups to different
    peers wait independently, so a slow peer never blocks another pair."""
    import threading

    def post(ops: List[Op]) -> object:
        works = []
        for send, peer, ptr, nbytes, *ch in ops:
            if nbytes == 0:
                continue
            t = _view(ptr, nbytes)
            tag = ch[0] if ch else 0  # independent matching order per channel, like one RCCL comm each
            works.append((t, dist.isend(t, peer, group=group, tag=tag) if send
                          else dist.irecv(t, peer, group=group, tag=tag)))
        done = threading.Event()
        if not works:
            done.set()
            return works, done, None

        def waiter() -> None:
            for _, w in works:
                w.wait()
            done.set()

        th = threading.Thread(target=waiter, daemon=True, name="akka-gloo-wait")
        th.start()
        return works, done, th

    def test(handle: object) -> bool:
        return handle[1].is_set()  # type: ignore[index]

    return post, test
