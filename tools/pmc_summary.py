#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc databases: per kernel, mean counter value per dispatch
(plus vgpr/lds/duration), for the kernels whose name matches an optional filter."""
import collections
import sqlite3
import sys


def main(dbs, filt=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for db in dbs:
        c = sqlite3.connect(db)
        q = ("select kernel_name, dispatch_id, counter_name, value, duration, vgpr_count, "
             "accum_vgpr_count, lds_block_size, grid_size, workgroup_size from counters_collection")
        per = collections.defaultdict(float)
        for name, did, cn, v, dur, vg, ag, lds, gs, wg in c.execute(q):
            if filt not in name:
                continue
            short = name.split("(")[0].replace("void ", "")
            per[(short, did, cn)] += v
            meta[short] = (vg, ag, lds, gs, wg)
            agg[short]["duration_ns"].append(dur)
        for (short, did, cn), v in per.items():
            agg[short][cn].append(v)
    for k, d in agg.items():
        vg, ag, lds, gs, wg = meta[k]
        print(f"== {k}  vgpr={vg} agpr={ag} lds={lds} grid={gs} wg={wg}")
        for cn, vals in sorted(d.items()):
            print(f"   {cn:28s} {sum(vals) / len(vals):16.1f}   (n={len(vals)})")


if __name__ == "__main__":
    args = sys.argv[1:]
    filt = ""
    if args and args[0].startswith("--filter="):
        filt = args.pop(0).split("=", 1)[1]
    main(args, filt)
