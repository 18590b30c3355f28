#!/usr/bin/env python3
"""Per-evaluation kernel breakdown of a rocprofv3 kernel-trace db of bench.py
(the last 1/NEVAL of the dispatches = one evaluation): total busy time, span,
and per-kernel count / total / average (us)."""
import collections
import re
import sqlite3
import sys

db = sys.argv[1]
neval = int(sys.argv[2]) if len(sys.argv) > 2 else 12
c = sqlite3.connect(db)
rows = list(c.execute("select name, queue_id, start, end from kernels order by start"))
n = len(rows) // neval
ev = rows[-n:]
busy = sum(e - s for _, _, s, e in ev) / 1e3
print(f"one eval: {n} dispatches, kernel sum {busy:.1f} us, span {(ev[-1][3] - ev[0][2]) / 1e3:.1f} us")
agg = collections.defaultdict(lambda: [0, 0.0])
for name, q, s, e in ev:
    nm = re.sub(r"\(.*", "", name.replace("void ", "").replace("(anonymous namespace)::", ""))
    agg[nm][0] += 1
    agg[nm][1] += (e - s) / 1e3
for k, (cnt, tot) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k[:48]:48s} n={cnt:4d} tot={tot:8.1f} avg={tot / cnt:7.1f}")
