#!/usr/bin/env python3
"""risk_accumulate measured AS AN OP, not HBM-resident.

Forms (ref ops/risk_accumulate.py:18-77; SURVEY §6 B6/B7 measured the reference op on
this host's CPU: 8.0 M values/s for ``values``, 5.4 M items/s for ``items``):

* ``values``: a JSON-decoded list of N numbers through ``risk_accumulate`` (native
  list pass), and the same including ``json.loads`` of the payload text;
* ``items``: N dicts with a ``risk`` field;
* ``csv``: ``source_uri`` + ``field`` — native row index + column parse, then the K12
  reduction on the GPU (H2D included) when one is present, else the CPU.

Prints one JSON line with values/s per form.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timed(fn, reps=3):
    best = float("inf")
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        best = min(best, time.perf_counter() - t0)
    return best, out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--csv-rows", type=int, default=10_000_000)
    a = ap.parse_args()
    from ops.risk_accumulate import risk_accumulate

    rng = random.Random(0)
    vals = [rng.uniform(-1000.0, 1000.0) for _ in range(a.n)]
    text = json.dumps({"values": vals})
    items = [{"id": i, "risk": v} for i, v in enumerate(vals)]
    res = {}
    os.environ["RISK_DEVICE"] = "auto"
    t, _ = timed(lambda: risk_accumulate({"values": vals}))
    res["values_op"] = round(a.n / t, 1)
    t, _ = timed(lambda: risk_accumulate(json.loads(text)))
    res["values_op_incl_json_decode"] = round(a.n / t, 1)
    t, _ = timed(lambda: risk_accumulate({"items": items}))
    res["items_op"] = round(a.n / t, 1)
    os.environ["RISK_NATIVE"] = "0"
    os.environ["RISK_DEVICE"] = "cpu"
    t, _ = timed(lambda: risk_accumulate({"values": vals}), reps=1)
    res["values_python_loop"] = round(a.n / t, 1)
    os.environ["RISK_NATIVE"] = "1"

    path = f"/tmp/atpu_risk_{a.csv_rows}.csv"
    if not os.path.exists(path):
        with open(path, "w") as f:
            f.write("id,risk\n")
            r = random.Random(1)
            f.writelines(f"{i},{r.uniform(-1000, 1000):.6f}\n" for i in range(a.csv_rows))
    try:
        import torch

        gpu = torch.cuda.is_available()
    except Exception:
        gpu = False
    os.environ["RISK_DEVICE"] = "gpu" if gpu else "cpu"
    payload = {"source_uri": path, "field": "risk", "start_row": 0, "shard_size": a.csv_rows}
    risk_accumulate(payload)  # builds / caches the row index (.rowidx) once
    t, out = timed(lambda: risk_accumulate(payload))
    res["csv_op"] = round(a.csv_rows / t, 1)
    res["csv_device"] = out.get("device", "cpu")
    print(json.dumps({"metric": "risk_accumulate op throughput (values/s)", "unit": "values/s",
                      "n": a.n, "csv_rows": a.csv_rows, "results": res,
                      "baseline": {"B6_values": 8.0e6, "B7_items": 5.4e6},
                      "vs_B6": round(res["values_op"] / 8.0e6, 2), "vs_B7": round(res["items_op"] / 5.4e6, 2)}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
