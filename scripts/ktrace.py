"""Per-kernel summary of rocprofv3 --kernel-trace CSV files (one per
process): calls, mean / median / min / max µs per kernel name, per file."""
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        continue
    by = {}
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or "?"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        by.setdefault(name, []).append(d)
    print(f"== {os.path.relpath(f, root)}")
    print("%-72s %6s %9s %9s %9s %9s" % ("kernel", "calls", "mean_us", "med_us", "min_us", "max_us"))
    for name, ds in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print("%-72s %6d %9.1f %9.1f %9.1f %9.1f" % (name[:72], len(ds), statistics.mean(ds), statistics.median(ds),
                                                     min(ds), max(ds)))
