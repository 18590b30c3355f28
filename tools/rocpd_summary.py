"""Summarise a rocprofv3 SQLite output: per-kernel count / total / avg (us)."""
import sqlite3, sys, glob, re
db = sys.argv[1]
if not db.endswith('.db'):
    db = glob.glob(db + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = 'name' if 'name' in cols else ('kernel_name' if 'kernel_name' in cols else cols[0])
rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start) from kernels group by {name_col} order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':70s} {'count':>7s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for n, cnt, s, a in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    n = re.sub(r'\(.*', '', n.replace('(anonymous namespace)::', '').replace('void ', ''))
    print(f"{n[:70]:70s} {cnt:7d} {s/1e6:10.3f} {a/1e3:9.2f} {100*s/tot:6.1f}")
print(f"TOTAL {tot/1e6:.3f} ms")
