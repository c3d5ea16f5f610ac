"""Summarise rocprofv3 counter-collection CSVs per kernel: mean counter values
and achieved bytes (FETCH_SIZE/WRITE_SIZE are KiB per dispatch).

usage: pmc_summary.py <dir-with-*_counter_collection.csv> [...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
                    short = name.split("(")[0].replace("void ", "")[:70]
                    key = (short, r.get("Grid_Size", ""))
                    try:
                        rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    except (KeyError, ValueError):
                        pass
    for (k, grid), cs in sorted(rows.items()):
        parts = []
        for c, v in sorted(cs.items()):
            med = sorted(v)[len(v) // 2]
            parts.append(f"{c}={sum(v) / len(v):.4g} (median {med:.4g}, n={len(v)})")
        print(f"{k} grid={grid}: " + " ".join(parts))


if __name__ == "__main__":
    main()
