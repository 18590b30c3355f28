#!/usr/bin/env python3
"""MFMA utilisation from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
SQ_WAVE_CYCLES GRBM_GUI_ACTIVE pass (tools/r02_measure.sh): per kernel family,
busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md, DVFS note),
plus the whole-run total over the sum of dispatch cycles.  Prints JSON."""
import collections
import json
import re
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
per = collections.defaultdict(lambda: collections.defaultdict(float))
for name, did, cn, v in c.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
    per[(name, did)][cn] += v
fam = collections.defaultdict(lambda: collections.defaultdict(float))
for (name, did), d in per.items():
    short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))
    f = fam[short]
    f["n"] += 1
    for k, v in d.items():
        f[k] += v
out = {}
tot_busy = tot_cyc = 0.0
for k, f in sorted(fam.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
    cyc = f["GRBM_GUI_ACTIVE"] / 8.0
    tot_busy += f["SQ_VALU_MFMA_BUSY_CYCLES"]
    tot_cyc += cyc
    out[k] = {"dispatches": int(f["n"]), "mfma_busy_frac": f["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc) if cyc else None,
              "gpu_cycles_per_dispatch": cyc / f["n"]}
print(json.dumps({"source": db, "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8)",
                  "all_kernels_mfma_busy_frac": tot_busy / (1024.0 * tot_cyc) if tot_cyc else None,
                  "kernels": out}, indent=1))
