#!/usr/bin/env python3
"""Phase markers of the last GP evaluation in a rocprofv3 kernel-trace db of
bench.py: start/end (us from the evaluation's first dispatch) of the marker
kernels, and the busy time per queue between consecutive markers."""
import re
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = list(c.execute("select name, queue_id, start, end from kernels order by start"))
names = [re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", "")) for n, *_ in rows]
starts = [i for i, n in enumerate(names) if n.startswith("k_gp_fwd")]
i0 = starts[-1]
t0 = rows[i0][2]
mark = ("k_gp_fwd", "k_add_diag_fwd", "k_check_symmetric", "k_chol_panel", "k_inv_double_diag", "k_trsv_persist",
        "k_mvn_rev", "k_tril_copy", "k_half_lower", "k_add_lower", "k_gp_rev_partials", "k_gp_rev_final")
for i in range(i0, len(rows)):
    n = names[i]
    if n.startswith(mark):
        print(f"{(rows[i][2] - t0) / 1e3:9.1f} {(rows[i][3] - t0) / 1e3:9.1f}  q{rows[i][1]}  {n[:40]}")
