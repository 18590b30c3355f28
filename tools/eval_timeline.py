#!/usr/bin/env python3
"""One evaluation's kernel timeline from a rocprofv3 kernel-trace db of the GP
bench: start / end offsets (us) from the evaluation's first kernel, duration
and queue.  eval_timeline.py DB [EVAL_INDEX] (evaluations are delimited by
k_gp_fwd*)."""
import re
import sqlite3
import sys

db = sys.argv[1]
e = int(sys.argv[2]) if len(sys.argv) > 2 else 4
c = sqlite3.connect(db)
rows = list(c.execute("select name, queue_id, start, end from kernels order by start"))
starts = [i for i, r in enumerate(rows) if "k_gp_fwd" in r[0]]
s, t = starts[e], (starts[e + 1] if e + 1 < len(starts) else len(rows))
t0 = rows[s][2]
for r in rows[s:t]:
    nm = re.sub(r"\(.*", "", r[0].replace("void ", "").replace("(anonymous namespace)::", ""))[:52]
    print(f"{nm:52s} q{r[1]} {(r[2] - t0) / 1e3:8.1f} {(r[3] - t0) / 1e3:8.1f} {(r[3] - r[2]) / 1e3:7.1f}")
print(f"span {(rows[t - 1][3] - t0) / 1e3:.1f} us")
