#!/usr/bin/env python3
"""Main-queue kernel time of one GP evaluation (the second-to-last complete
one in a rocprofv3 kernel-trace db of bench.py) split into phases:
pre (before the first panel), forward (first panel .. last panel, main
queue), mid (after the last panel .. the MVN reverse), reverse (Murray) and
post; plus the other queues' busy time."""
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, queue_id, start, end from kernels order by start"))
names = [re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", "")) for n, *_ in rows]
st = [i for i, n in enumerate(names) if n.startswith("k_gp_fwd")]
a, b = st[-3], st[-2]
ev = list(zip(names[a:b], rows[a:b]))
q0 = ev[0][1][1]
panels = [i for i, (n, r) in enumerate(ev) if n == "k_chol_panel"]
mvnrev = [i for i, (n, r) in enumerate(ev) if n.startswith("k_mvn_rev")][0]
addl = [i for i, (n, r) in enumerate(ev) if n.startswith("k_add_lower")][-1]
cuts = {"pre": (0, panels[0]), "forward": (panels[0], panels[-1] + 1), "mid": (panels[-1] + 1, mvnrev + 1),
        "reverse": (mvnrev + 1, addl), "post": (addl, len(ev))}
t0 = ev[0][1][2]
tot = 0
for k, (i, j) in cuts.items():
    main = [r for n, r in ev[i:j] if r[1] == q0]
    busy = sum(e - s for _, _, s, e in main) / 1e3
    span = ((ev[j - 1][1][3] - ev[i][1][2]) / 1e3) if j > i else 0
    tot += busy
    print(f"{k:8s} main busy {busy:7.1f} us  span {span:7.1f} us  kernels {len(main)}")
other = sum((r[3] - r[2]) for n, r in ev if r[1] != q0) / 1e3
print(f"total main busy {tot:.1f} us, eval span {(ev[-1][1][3] - t0) / 1e3:.1f} us, other queues busy {other:.1f} us")

# per-kernel totals of the chosen evaluation (all queues), largest first
agg = {}
for n, r in ev:
    k = re.sub(r"<.*", "", n) if len(sys.argv) < 3 else n
    t, c_ = agg.get(k, (0.0, 0))
    agg[k] = (t + (r[3] - r[2]) / 1e3, c_ + 1)
for k, (t, c_) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"  {t:8.1f} us  {c_:4d}  {k}")
