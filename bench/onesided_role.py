"""Reduce role of the one-sided lane alone (csrc/kernels/onesided.hip,
onesided_reduce_role_bench): one process, local windows, every chunk decided
with all N sources and every peer gated, so each piece reads N x its span and
writes its span to the output + N-1 gather rows.  One JSON line per case:
ms per launch and TB/s of (N read + N written) x block bytes.

    python bench/onesided_role.py --n 2,4,8 --block-mb 32 --threads 256,1024 --grid 256,512
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="2,4,8")
    ap.add_argument("--block-mb", type=float, default=32.0)
    ap.add_argument("--chunk-mb", type=float, default=4.0)
    ap.add_argument("--part-kb", type=float, default=256.0)
    ap.add_argument("--nsub", default="0", help="pieces per part (0: enough for --grid)")
    ap.add_argument("--threads", default="256,1024")
    ap.add_argument("--grid", default="256")
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from akka_allreduce_amd._native_loader import load

    nat = load()
    es = 4 if a.dtype == "float32" else 2
    block = int(a.block_mb * (1 << 20)) // es
    chunk = int(a.chunk_mb * (1 << 20)) // es
    part = int(a.part_kb * 1024) // es
    for n in [int(v) for v in a.n.split(",")]:
        for nt in [int(v) for v in a.threads.split(",")]:
            for grid in [int(v) for v in a.grid.split(",")]:
                for ns in [int(v) for v in a.nsub.split(",")]:
                    k = (block + chunk - 1) // chunk
                    p = (chunk + part - 1) // part
                    nsub = ns if ns > 0 else max(1, min(part // 4096, -(-grid // (k * p))))
                    ms = nat.onesided_reduce_role_bench(n, block, chunk, part, nsub, a.dtype, nt, grid, a.iters, 0)
                    moved = 2 * n * block * es
                    print(json.dumps({"N": n, "block_mb": a.block_mb, "threads": nt, "grid": grid, "nsub": nsub,
                                      "dtype": a.dtype, "ms": round(ms, 4),
                                      "TBps_traffic": round(moved / (ms * 1e-3) / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
