"""HIP API calls per round from rocprofv3 --hip-trace CSVs (one per process):
count and median duration of every function, divided by the launches of the
round's main kernel (ipc / one-sided round kernel) in the same process.

    python scripts/r06/api_per_round.py <trace dir>
"""
import csv
import glob
import os
import re
import statistics
import sys

MAIN = re.compile(r"ipc_(?!round_bump)\w*kernel|os_round_kernel|reduce_\w*kernel")


def main():
    d = sys.argv[1]
    for kf in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        af = kf.replace("kernel_trace.csv", "hip_api_trace.csv")
        if not os.path.exists(af):
            continue
        rounds = sum(1 for r in csv.DictReader(open(kf)) if MAIN.search(r.get("Kernel_Name", "")))
        calls: dict = {}
        for r in csv.DictReader(open(af)):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            calls.setdefault(r["Function"], []).append(dur)
        print(f"{os.path.basename(kf)}: {rounds} round kernels")
        top = sorted(calls.items(), key=lambda kv: -len(kv[1]))[:14]
        for name, v in top:
            print(f"  {name:34s} per_round {len(v) / max(1, rounds):7.2f}  median_us {statistics.median(v):8.2f}")


if __name__ == "__main__":
    main()
