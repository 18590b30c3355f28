#!/usr/bin/env python3
"""Decode the chain workgroup's event log printed by tools/ubench_panel:
per-step phase durations (us) between consecutive events."""
import re
import sys

txt = open(sys.argv[1]).read()
for line in txt.splitlines():
    if not line.startswith("WG 0:"):
        continue
    ev = [(int(j), int(t), int(p), float(us)) for j, t, p, us in re.findall(r"\[j(\d+) t(\d+) p(\d+) ([\d.]+)us\]", line)]
    names = {2: "start", 10: "factor+leaves", 3: "Dinv st", 4: "publish", 11: "wait+load", 12: "lstore", 13: "TRSM", 9: "SYRK"}
    prev = None
    for j, t, p, us in ev:
        if prev is not None:
            print(f"  j{j} {names.get(p, p):>10s} +{us - prev:6.2f}")
        prev = us
        if p == 2:
            print(f"step {j} at {us:.2f}")
