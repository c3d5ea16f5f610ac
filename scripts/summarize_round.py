"""Summary of bench/onesided_round.py rank files: the slowest rank per case."""
import json
import sys

d, n = sys.argv[1], int(sys.argv[2])
rows = [json.load(open(f"{d}/rank{i}.json")) for i in range(n)]
for j, c in enumerate(rows[0]["cases"]):
    ms = max(r["cases"][j].get("ms", 0.0) for r in rows)
    line = {"lane": c["lane"], "size_mb": c["size_mb"], "exact": all(r["cases"][j].get("exact") for r in rows),
            "max_ms": round(ms, 4), "algbw_GBps": round(c["size_mb"] * 2 ** 20 / (ms * 1e-3) / 1e9, 1) if ms else None}
    if c.get("exception"):
        line["exception"] = c["exception"]
    if c.get("info"):
        line["info"] = {k: c["info"].get(k) for k in ("threads", "role_wgs", "pieces_per_part", "ranks_on_this_gpu")}
    print(json.dumps(line))
if "cfg4" in rows[0]:
    print(json.dumps(rows[0]["cfg4"]))
