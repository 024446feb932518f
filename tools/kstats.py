#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 results database: tools/kstats.py DB [topN]."""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3 from kernels group by name "
                 "order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel time {tot:.2f} ms over {sum(r[1] for r in rows)} dispatches")
print(f"{'ms':>9} {'%':>6} {'calls':>7} {'avg us':>9}  kernel")
for r in rows[:top]:
    name = r[0].replace("atpu::(anonymous namespace)::", "").replace("bool _Accum", "bf16")
    print(f"{r[2]:9.2f} {100 * r[2] / tot:6.1f} {r[1]:7d} {r[3]:9.1f}  {name[:120]}")
