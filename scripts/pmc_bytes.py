"""Bytes moved per chunk-reduce dispatch from raw TCC/EA request counters.

read  = 128 * TCC_EA0_RDREQ_128B + 64 * TCC_EA0_RDREQ_64B + 32 * TCC_EA0_RDREQ_32B
write = 64 * TCC_EA0_WRREQ_64B + 32 * (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)
The same workload runs once per counter pass, so the k-th reduce dispatch of
every pass is the same launch: passes are joined on that index, and
consecutive dispatches of one kernel/grid form one configuration (1 warm-up +
timed iterations).  Reported per configuration: mean read / write MiB per
dispatch (write = the chunk, read should be nsrc x chunk), the share of EA
reads that went to DRAM, the derived FETCH_SIZE (which counts a 128-B
request as 64 B unless TCC_BUBBLE sees it) and kernel time from the trace.

usage: pmc_bytes.py <pass dir> [...]
"""
import collections
import csv
import glob
import os
import re
import sys


def load(d):
    """-> list (dispatch order) of (kernel, grid, {counter: value}, duration_ns)"""
    disp = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
                if "reduce_" not in name:
                    continue
                did = int(r["Dispatch_Id"])
                e = disp.setdefault(did, [name.split("(")[0].replace("void akka::", ""), int(r["Grid_Size"]), {}, 0])
                e[2][r["Counter_Name"]] = float(r["Counter_Value"])
                e[3] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [disp[k] for k in sorted(disp)]


def main():
    passes = [load(d) for d in sys.argv[1:]]
    n = min(len(p) for p in passes)
    rows = []
    for i in range(n):
        k, g = passes[0][i][0], passes[0][i][1]
        cs = {}
        for p in passes:
            cs.update(p[i][2])
        rows.append((k, g, cs, passes[0][i][3]))
    groups = []
    for k, g, cs, t in rows:
        if groups and groups[-1][0] == (k, g):
            groups[-1][1].append((cs, t))
        else:
            groups.append(((k, g), [(cs, t)]))
    print(f"{'kernel':36s} {'nsrc':>4s} {'chunk MiB':>9s} {'RD MiB':>9s} {'RD/chunk':>8s} {'DRAM%':>6s} "
          f"{'FETCH_SIZE MiB':>14s} {'us':>8s} {'TB/s':>6s}")
    for (k, g), its in groups:
        timed = its[1:] or its  # drop the warm-up dispatch
        m = collections.defaultdict(float)
        for cs, _ in timed:
            for c, v in cs.items():
                m[c] += v / len(timed)
        if "TCC_EA0_RDREQ_128B_sum" not in m:
            continue
        rd = 128 * m["TCC_EA0_RDREQ_128B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 32 * m["TCC_EA0_RDREQ_32B_sum"]
        wr = 64 * m["TCC_EA0_WRREQ_64B_sum"] + 32 * (m["TCC_EA0_WRREQ_sum"] - m["TCC_EA0_WRREQ_64B_sum"])
        dram = 100.0 * m["TCC_EA0_RDREQ_DRAM_sum"] / max(1.0, m["TCC_EA0_RDREQ_sum"])
        fetch = m.get("FETCH_SIZE", float("nan")) / 1024
        us = sorted(t for _, t in timed)[len(timed) // 2] / 1e3
        nsrc = re.search(r"<[^,]+, (\d+)", k)
        print(f"{k[:36]:36s} {nsrc.group(1) if nsrc else '?':>4s} {wr / 2**20:9.2f} {rd / 2**20:9.2f} "
              f"{rd / max(wr, 1):8.3f} {dram:6.1f} {fetch:14.2f} {us:8.2f} {(rd + wr) / (us * 1e-6) / 1e12:6.2f}")


if __name__ == "__main__":
    main()
