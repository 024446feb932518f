#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 ``--pmc`` counter CSV: tools/pmc_summ.py <dir or csv> [--match SUBSTR].

For every kernel: dispatches, mean duration (us), the mean of each counter per dispatch, and the
derived L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS)) and effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md "DVFS give-back") when present."""
import argparse
import collections
import csv
import glob
import os


def load(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
        if not cands:
            raise SystemExit(f"no counter_collection.csv under {path}")
        path = cands[0]
    return list(csv.DictReader(open(path)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = load(a.path)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in rows:
        name = r.get("Kernel_Name", "")
        if a.match and a.match not in name:
            continue
        did = r.get("Dispatch_Id")
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        try:
            dur[name][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        except (KeyError, ValueError):
            pass
    tot = {k: sum(v.values()) for k, v in dur.items()}
    for name in sorted(per, key=lambda k: -tot.get(k, 0.0))[:a.top]:
        c = per[name]
        n = len(dur[name]) or 1
        d = sum(dur[name].values()) / n if dur[name] else float("nan")
        mean = {k: sum(v) / len(v) for k, v in c.items()}
        extra = []
        if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
            h, m = mean["TCC_HIT_sum"], mean["TCC_MISS_sum"]
            extra.append(f"L2hit={100 * h / max(1.0, h + m):.1f}%")
        if "GRBM_GUI_ACTIVE" in mean and d == d and d > 0:
            extra.append(f"clk={mean['GRBM_GUI_ACTIVE'] / 8 / d / 1e3:.2f}GHz")
        short = name.replace("atpu::(anonymous namespace)::", "")[:90]
        print(f"{n:5d} x {d:9.1f} us  {short}")
        print("        " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(mean.items())) + ("  " + " ".join(extra)))


if __name__ == "__main__":
    main()
