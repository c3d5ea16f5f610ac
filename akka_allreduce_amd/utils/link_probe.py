"""Per-link bandwidth matrix of the job's ranks (csrc/transport/link_probe.h).

``probe_links`` measures, for every ordered pair (src, dst), src writing a
buffer into dst's mapped memory (push) and src reading dst's (pull) while
every other rank is idle, then every rank pushing to all its peers at once
(the direct algorithm's traffic pattern).  On an MI355X node the pairs are
xGMI links -- SURVEY §5.8 assumes ~153 GB/s each, the bench's analytic bound
``algbw <= N * L / 2`` uses that figure; this is the measurement.  Ranks
sharing one GPU (rehearsal) or CPU ranks (shared memory) exercise the flow
but measure no link.

Collective: every rank calls it, in the same order (handles exchanged and
pairs sequenced over torch.distributed, gloo is enough).
"""
from __future__ import annotations

from typing import Optional

import torch


def probe_links(rank: int, world: int, device: torch.device, mib: float = 64.0, iters: int = 3) -> Optional[dict]:
    """Returns the matrices on rank 0 (None elsewhere): GB/s, row = source."""
    import torch.distributed as dist

    from .._native_loader import load

    n = load()
    dev_index = device.index if device.type == "cuda" else -1
    if device.type == "cuda" and dev_index is None:
        dev_index = torch.cuda.current_device()
    nbytes = int(mib * (1 << 20)) // 16 * 16
    p = n.LinkProbe(dev_index, rank, world, nbytes)
    handles = [None] * world
    dist.all_gather_object(handles, p.handle())
    p.open(handles)
    dist.barrier()
    p.unlink()
    push = [None] * world
    pull = [None] * world
    for src in range(world):
        for dst in range(world):
            if src == dst:
                continue
            dist.barrier()  # one pair at a time: every other rank idle
            if rank == src:
                push[dst] = round(nbytes * iters / p.push([dst], iters) / 1e9, 2)
                pull[dst] = round(nbytes * iters / p.pull([dst], iters) / 1e9, 2)
    dist.barrier()
    peers = [q for q in range(world) if q != rank]
    t = p.push(peers, iters)  # every rank at once: the direct algorithm's pattern
    all_push = round(nbytes * iters * len(peers) / t / 1e9, 2)
    dist.barrier()
    t = p.pull(peers, iters)
    all_pull = round(nbytes * iters * len(peers) / t / 1e9, 2)
    rows = [None] * world
    dist.all_gather_object(rows, (push, pull, all_push, all_pull))
    del p
    if rank != 0:
        return None
    return {
        "bytes_per_copy": nbytes,
        "iters": iters,
        "push_GBps": [r[0] for r in rows],   # [src][dst], remote writes by src
        "pull_GBps": [r[1] for r in rows],   # [src][dst], src reads dst's memory
        "all_peers_push_GBps_per_rank": [r[2] for r in rows],
        "all_peers_pull_GBps_per_rank": [r[3] for r in rows],
    }
