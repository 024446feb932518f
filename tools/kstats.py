#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 run.

  tools/kstats.py DB.db [topN]            results database (sqlite)
  tools/kstats.py --csv kernel_stats.csv [topN]
"""
import csv
import sqlite3
import sys


def rows_db(path):
    c = sqlite3.connect(path)
    return c.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3 from kernels group by name "
                     "order by 3 desc").fetchall()


def rows_csv(path):
    out = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3)
           for r in csv.DictReader(open(path))]
    return sorted(out, key=lambda r: -r[2])


def main(argv):
    if argv[0] == "--csv":
        rows, argv = rows_csv(argv[1]), argv[2:]
    else:
        rows, argv = rows_db(argv[0]), argv[1:]
    top = int(argv[0]) if argv else 25
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot:.2f} ms over {sum(r[1] for r in rows)} dispatches")
    print(f"{'ms':>9} {'%':>6} {'calls':>7} {'avg us':>9}  kernel")
    for r in rows[:top]:
        name = r[0].replace("atpu::(anonymous namespace)::", "").replace("bool _Accum", "bf16")
        print(f"{r[2]:9.2f} {100 * r[2] / max(tot, 1e-9):6.1f} {r[1]:7d} {r[3]:9.1f}  {name[:120]}")


if __name__ == "__main__":
    main(sys.argv[1:])
