#!/usr/bin/env python3
"""Summarise a rocprofv3 .db (kernel trace): per-kernel stats + tail of the timeline."""
import sqlite3
import sys

db = sys.argv[1]
tail = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = sqlite3.connect(db)
print("%-70s %6s %10s %10s" % ("kernel", "calls", "total_us", "avg_us"))
for name, calls, tot in c.execute(
        "select name, count(*), sum(end-start)/1000.0 from kernels group by name order by sum(end-start) desc limit 15"):
    print("%-70s %6d %10.1f %10.2f" % (name[:70], calls, tot, tot / calls))
rows = list(c.execute("select name, start, end, stream_id from kernels order by start"))
if rows:
    t0 = rows[-tail][1] if len(rows) >= tail else rows[0][1]
    print("\ntimeline (last %d dispatches, us from first shown): name start dur gap stream" % tail)
    prev = None
    for n, s, e, st in rows[-tail:]:
        gap = (s - prev) / 1e3 if prev else 0.0
        print("  %-50s %10.1f %8.2f %8.2f %s" % (n[:50], (s - t0) / 1e3, (e - s) / 1e3, gap, st))
        prev = e
