#!/usr/bin/env python3
"""HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_traffic.sh, calibrated on a known 8-byte-per-lane stream
(tools/calib_fetch.hip: 1 GiB read and written), per the guide's rule that
non-16-B access widths must be calibrated.  Prints JSON for profiles/."""
import collections
import glob
import json
import sqlite3
import sys

TAG = sys.argv[1] if len(sys.argv) > 1 else "r01"
BASE = "gpurun_out/pmc_%s_%s/run_results.db"


def per_kernel(name):
    """kernel short name -> list of per-dispatch counter totals (KB as reported)"""
    dbs = glob.glob(BASE % (TAG, name)) or glob.glob(f"gpurun_out/pmc_{TAG}_{name}/*/*.db")
    out = collections.defaultdict(dict)
    for db in dbs:
        c = sqlite3.connect(db)
        for kn, did, v in c.execute("select kernel_name, dispatch_id, value from counters_collection"):
            short = kn.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            out[short][did] = out[short].get(did, 0.0) + v
    return {k: list(v.values()) for k, v in out.items()}


def mean(x):
    return sum(x) / len(x) if x else 0.0


calib_bytes = float(1 << 30)
f = per_kernel("calib_fetch")
w = per_kernel("calib_write")
rf = calib_bytes / (mean(f["k_read8"]) * 1024.0)   # true bytes per reported byte (FETCH_SIZE in KB)
rw = calib_bytes / (mean(w["k_write8"]) * 1024.0)
res = {"calibration": {"kernel": "tools/calib_fetch.hip (8 B/lane, 1 GiB)", "fetch_scale": rf,
                       "write_scale": rw}}
for wl, kern in (("glm", "k_glm_reg"), ("gp", "k_gemm")):
    fk, wk = per_kernel(f"{wl}_fetch"), per_kernel(f"{wl}_write")
    fv = [v for k, vs in fk.items() if k.startswith(kern) for v in vs]
    wv = [v for k, vs in wk.items() if k.startswith(kern) for v in vs]
    res[wl] = {"kernel": kern + "*", "launches": len(fv),
               "fetch_bytes_per_launch": mean(fv) * 1024.0 * rf,
               "write_bytes_per_launch": mean(wv) * 1024.0 * rw}
    res[wl]["traffic_bytes_per_launch"] = res[wl]["fetch_bytes_per_launch"] + res[wl]["write_bytes_per_launch"]
print(json.dumps(res, indent=1))
