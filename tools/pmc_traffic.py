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
def per_dispatch(name):
    """[(kernel short name, grid x, fetch-or-write KB)] per dispatch"""
    dbs = glob.glob(BASE % (TAG, name)) or glob.glob(f"gpurun_out/pmc_{TAG}_{name}/*/*.db")
    out = collections.defaultdict(float)
    meta = {}
    for db in dbs:
        c = sqlite3.connect(db)
        try:
            rows = c.execute("select kernel_name, dispatch_id, grid_size_x, value from counters_collection").fetchall()
        except sqlite3.OperationalError:
            rows = [(kn, did, 0, v) for kn, did, v in
                    c.execute("select kernel_name, dispatch_id, value from counters_collection")]
        for kn, did, gx, v in rows:
            out[did] += v
            meta[did] = (kn.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0], gx)
    return [(meta[d][0], meta[d][1], out[d]) for d in sorted(out)]


for wl, kern in (("glm", "k_glm_reg"), ("gp", "k_gemm")):
    fk, wk = per_kernel(f"{wl}_fetch"), per_kernel(f"{wl}_write")
    fv = [v for k, vs in fk.items() if k.startswith(kern) for v in vs]
    wv = [v for k, vs in wk.items() if k.startswith(kern) for v in vs]
    res[wl] = {"kernel": kern + "*", "launches": len(fv),
               "fetch_bytes_per_launch": mean(fv) * 1024.0 * rf,
               "write_bytes_per_launch": mean(wv) * 1024.0 * rw}
    res[wl]["traffic_bytes_per_launch"] = res[wl]["fetch_bytes_per_launch"] + res[wl]["write_bytes_per_launch"]
# round 4: the dominant kernel (k_chol_panel) and the largest K^{-1} share
# (C += W_k^T W_k of the last block row: k_gemm TN lower, the widest grid),
# each beside its algorithmic bytes (N = 4096, 512-column panels)
if glob.glob(BASE % (TAG, "gp_fetch")):
    N, P = 4096, 512
    fd, wd = per_dispatch("gp_fetch"), per_dispatch("gp_write")
    pf = [v for k, g, v in fd if k.startswith("k_chol_panel")]
    pw = [v for k, g, v in wd if k.startswith("k_chol_panel")]
    # a panel reads its (N - J) x 512 columns and writes the factor back: 16 (N - J) 512 B, mean over the 8 panels
    alg_panel = sum(16.0 * (N - J) * P for J in range(0, N, P)) / (N // P)
    res["k_chol_panel"] = {"launches": len(pf), "fetch_bytes_per_launch": mean(pf) * 1024.0 * rf,
                           "write_bytes_per_launch": mean(pw) * 1024.0 * rw, "algorithmic_bytes_per_launch": alg_panel}
    res["k_chol_panel"]["waste_ratio"] = (res["k_chol_panel"]["fetch_bytes_per_launch"] +
                                          res["k_chol_panel"]["write_bytes_per_launch"]) / alg_panel
    # the share with the most 64 x 64 tiles (grid_x counts threads: 256 per workgroup, 512 for the 8-wave
    # ", 2>" variant; until round 6 the widest grid was taken, which picked the 8-wave share of row 5)
    def tiles(k, g):
        return g // (512 if k.rstrip().endswith("2>") else 256)
    share = [(tiles(k, g), v) for k, g, v in fd if k.startswith("k_gemm<64, 64, 16, true, false, 1")]
    sharew = [(tiles(k, g), v) for k, g, v in wd if k.startswith("k_gemm<64, 64, 16, true, false, 1")]
    if share:
        tmax = max(t for t, v in share)
        f1 = [v for t, v in share if t == tmax]
        w1 = [v for t, v in sharew if t == tmax]
        r1 = 64 * int(round(((8 * tmax + 1) ** 0.5 - 1) / 2))  # tmax = T (T + 1) / 2 tiles, C is r1 x r1 lower
        # W_k (512 x r1) read + C's lower triangle (r1 (r1 + 1) / 2) read and written
        alg_share = 8.0 * (P * r1 + r1 * (r1 + 1))
        res["k_gemm_share_last"] = {"tiles": tmax, "rows": r1, "launches": len(f1),
                                    "fetch_bytes_per_launch": mean(f1) * 1024.0 * rf,
                                    "write_bytes_per_launch": mean(w1) * 1024.0 * rw,
                                    "algorithmic_bytes_per_launch": alg_share}
        res["k_gemm_share_last"]["waste_ratio"] = (res["k_gemm_share_last"]["fetch_bytes_per_launch"] +
                                                   res["k_gemm_share_last"]["write_bytes_per_launch"]) / alg_share
print(json.dumps(res, indent=1))
