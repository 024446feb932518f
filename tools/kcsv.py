#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --stats CSV: tools/kcsv.py run_kernel_stats.csv [topN] [title]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
if len(sys.argv) > 3:
    print("#", sys.argv[3])
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
print(f"{'ms':>9} {'%':>6} {'calls':>7} {'avg us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    name = r["Name"].replace("atpu::(anonymous namespace)::", "").replace("bool _Accum", "bf16")
    t = float(r["TotalDurationNs"]) / 1e6
    print(f"{t:9.2f} {100 * t * 1e6 / tot:6.1f} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:9.1f}  {name[:110]}")
