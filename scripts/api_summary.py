#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--hip-trace`` CSV: calls and host time per HIP API
function, divided by a round count, to see what the host issues per round.

usage: api_summary.py <dir with *_hip_api_trace.csv> [rounds]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*_hip_api_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        n = r.get("Function", r.get("Operation", "?"))
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[n][0] += 1
        tot[n][1] += t
    print(f"{'function':40} {'calls':>7} {'per_round':>9} {'total_us':>10} {'avg_us':>8}")
    for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:30]:
        print(f"{n[:40]:40} {c:7d} {c / rounds:9.2f} {t:10.1f} {t / c:8.2f}")


if __name__ == "__main__":
    main()
