#!/usr/bin/env python3
"""Print a window of the rocprofv3 kernel timeline (per queue) from a rocpd db:
start offset (us), duration (us), gap to the previous kernel on the same queue."""
import sqlite3
import sys

db = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 60
c = sqlite3.connect(db)
rows = list(c.execute("select name, queue_id, start, end from kernels order by start"))
t0 = rows[skip][2]
last = {}
for name, q, s, e in rows[skip:skip + count]:
    short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
    gap = (s - last[q]) / 1e3 if q in last else 0.0
    last[q] = e
    print(f"q{q:<3d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap:6.1f}  {short}")
