"""Per-round timeline of exact ipc rounds from rocprofv3 --kernel-trace CSVs
(one file per process): engine path vs direct launch, kernel by kernel.

The main kernel of a round is the ipc / one-sided round kernel.  Launches of
it are split into runs (consecutive launches less than --split-ms apart: the
barriers between the cases of bench/onesided_round.py are longer); per run of
at least --min-rounds launches:
  period_us   median start-to-start interval of the main kernel
  kernel_us   median duration of the main kernel
  gap_us      median idle time between one main kernel's end and the next start
  between     every other kernel launched in those gaps: calls per round and
              median duration (the engine path's counts fill / poison / ...)
Runs are listed in time order (bench/onesided_round.py: one run per size,
in --sizes-mb order; its warm-up launches fall below --min-rounds).

    python scripts/engine_path_trace.py <trace dir> [--split-ms 3] [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

MAIN = re.compile(r"ipc_(?!round_bump)\w*kernel|os_round_kernel")


def runs_of(rows, split_ns, min_rounds):
    mains = [r for r in rows if MAIN.search(r["name"])]
    runs, cur = [], []
    for r in mains:
        if cur and r["start"] - cur[-1]["end"] > split_ns:
            runs.append(cur)
            cur = []
        cur.append(r)
    if cur:
        runs.append(cur)
    return [run for run in runs if len(run) >= min_rounds]


def summarize(rows, run):
    per, dur, gap = [], [], []
    between: dict = {}
    for a, b in zip(run, run[1:]):
        per.append((b["start"] - a["start"]) / 1e3)
        gap.append((b["start"] - a["end"]) / 1e3)
        for r in rows:
            if a["end"] <= r["start"] < b["start"] and not MAIN.search(r["name"]):
                between.setdefault(r["name"], []).append((r["end"] - r["start"]) / 1e3)
    dur = [(r["end"] - r["start"]) / 1e3 for r in run]
    n = max(1, len(run) - 1)
    out = {"rounds": len(run), "main": run[0]["name"][:60], "period_us": round(statistics.median(per), 1),
           "kernel_us": round(statistics.median(dur), 1), "gap_us": round(statistics.median(gap), 1),
           "between": {k[:60]: {"per_round": round(len(v) / n, 2), "median_us": round(statistics.median(v), 1)}
                       for k, v in sorted(between.items())}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--split-ms", type=float, default=3.0)
    ap.add_argument("--min-rounds", type=int, default=6)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    res = {}
    for f in sorted(glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True)):
        rows = []
        for r in csv.DictReader(open(f)):
            rows.append({"name": r.get("Kernel_Name") or r.get("KernelName") or "?",
                         "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"])})
        rows.sort(key=lambda r: r["start"])
        res[os.path.relpath(f, a.root)] = [summarize(rows, run) for run in runs_of(rows, a.split_ms * 1e6,
                                                                                    a.min_rounds)]
    for f, runs in res.items():
        print(f"== {f}")
        for i, s in enumerate(runs):
            print(f"  run {i}: rounds {s['rounds']:3d} period {s['period_us']:8.1f} us  kernel "
                  f"{s['kernel_us']:8.1f}  gap {s['gap_us']:7.1f}  {s['main']}")
            for k, v in s["between"].items():
                print(f"      {v['per_round']:5.2f}/round {v['median_us']:7.1f} us  {k}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
