"""Bandwidth of the exact ipc round's reduce role alone (csrc/kernels/ipc.hip,
ipc_reduce_role_bench): one process, local fine-grained windows with every
push flag pre-set, so the kernel only waits zero times and sums.  Bytes per
launch: N x block read (N-1 window slots + the rank's own input) + 2 x block
written (output block + `reduced` row, pull mode).  Compares system-coherent
slot loads (sc0 sc1, the default) with plain loads behind the acquire.

    python bench/ipc_reduce_role.py [--n 2,4,8] [--block-mb 4,32] [--threads 256,1024]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="2,4,8")
    ap.add_argument("--block-mb", default="4,32")
    ap.add_argument("--threads", default="256,1024")
    ap.add_argument("--modes", default="sys,plain,lite", help="sys: sc0 sc1 slot loads + fences; plain: plain slot "
                    "loads behind the acquire; lite: sc loads, write-through window stores, no fences")
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kinds", default="fine", help="window memory: fine,coarse,uncached")
    ap.add_argument("--portion-kb", default="512", help="portion sizes (KiB): 4 reduce workgroups per portion")
    ap.add_argument("--max-wgs", default="1024", help="grid caps, in 256-thread workgroups (AKKA_IPC_MAX_WGS)")
    a = ap.parse_args()
    from akka_allreduce_amd._native_loader import load

    n = load()
    es = 4 if a.dtype == "float32" else 2
    for N in [int(x) for x in a.n.split(",")]:
        for mb in [float(x) for x in a.block_mb.split(",")]:
            block = int(mb * (1 << 20)) // es
            for kind in a.kinds.split(","):
                for pk in [int(x) for x in a.portion_kb.split(",")]:
                    for th in [int(x) for x in a.threads.split(",")]:
                        for cap in [int(x) for x in a.max_wgs.split(",")]:
                            for mode in a.modes.split(","):
                                ms = n.ipc_reduce_role_bench(N, block, pk << 10, a.dtype, mode == "plain", a.iters,
                                                             th, 0, kind, mode == "lite", cap)
                                rd, wr = N * block * es, 2 * block * es
                                print(json.dumps({"N": N, "block_mb": mb, "kind": kind, "portion_kb": pk,
                                                  "threads": th, "max_wgs": cap, "loads": mode, "dtype": a.dtype,
                                                  "us": round(ms * 1e3, 2), "read_bytes": rd, "write_bytes": wr,
                                                  "TBps": round((rd + wr) / (ms * 1e-3) / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
