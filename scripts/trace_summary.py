#!/usr/bin/env python3
"""Summarise rocprofv3 CSV traces (kernel + memory copy): per-name totals and
busy time per queue/stream, to see what a round spends its GPU time on.

usage: trace_summary.py <dir with *_kernel_trace.csv / *_memory_copy_trace.csv>
"""
import collections
import csv
import glob
import os
import sys


def load(d, kind):
    rows = []
    for f in glob.glob(os.path.join(d, "**", f"*_{kind}.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    d = sys.argv[1]
    ks = load(d, "kernel_trace")
    ms = load(d, "memory_copy_trace")
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in ks:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:60]
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[("kernel", n)][0] += 1
        tot[("kernel", n)][1] += t
    for r in ms:
        n = f'{r.get("Direction", "?")} {r.get("Src_Agent_Id", "")}->{r.get("Dst_Agent_Id", "")}'
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[("copy", n)][0] += 1
        tot[("copy", n)][1] += t
    print(f"{'kind':7} {'name':62} {'calls':>6} {'total_us':>10} {'avg_us':>9}")
    for (k, n), (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:25]:
        print(f"{k:7} {n:62} {c:6d} {t:10.1f} {t / c:9.2f}")
    allr = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks + ms]
    if allr:
        allr.sort()
        span = (allr[-1][1] - allr[0][0]) / 1e3
        busy, cur_s, cur_e = 0, None, None
        for s, e in allr:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        print(f"\nspan {span:.1f} us, GPU busy (union of kernels+copies) {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
