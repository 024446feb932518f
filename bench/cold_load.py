#!/usr/bin/env python3
"""Cold model load, end to end, in a fresh process on one GPU.

What an LRU miss costs the agent (ref ``ops/_tpu_runtime.py:34-63`` builds its handle on a
miss): for each classify model, a ``map_classify`` CSV job on a model the cache does not
hold, against the same job once the model is resident; the handle's phases
(``weights_ms``: seeded init on the device, or a safetensors load + H2D; ``engine_ms``:
LN folding, buffers, graph capture). The HIP context is created first and timed alone.
Summarize models: ``build_model`` + engine. ``--h2d`` adds the first-copy probe: a 219 MB
pageable host buffer copied to HBM in this fresh process, first vs later copies.
One JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def emit(obj):
    print(json.dumps(obj), flush=True)


def ms(t0):
    return round((time.perf_counter() - t0) * 1e3, 2)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--classify", default="bert-base,bert-large")
    ap.add_argument("--summarize", default="t5-base,bart-large-cnn")
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--h2d", action="store_true")
    a = ap.parse_args()
    import torch

    t0 = time.perf_counter()
    dev = torch.device("cuda", 0)
    torch.empty(1, device=dev)
    torch.cuda.synchronize(dev)
    emit({"what": "hip_context_ms", "ms": ms(t0)})
    if a.h2d:
        # where the first-copy cost of a fresh process comes from: a 4 KiB copy first, then
        # buffer A twice, then a second, freshly written buffer B of the same size
        n = 219_212_032
        srcs = {"A": torch.empty(n, dtype=torch.uint8).random_(0, 255),
                "B": torch.empty(n, dtype=torch.uint8).random_(0, 255)}
        small = torch.ones(4096, dtype=torch.uint8)
        for name, src in (("tiny", small), ("A", srcs["A"]), ("A", srcs["A"]), ("B", srcs["B"])):
            dst = torch.empty(src.numel(), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            dst.copy_(src)
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            emit({"what": "h2d_pageable", "src": name, "bytes": src.numel(), "ms": round(el * 1e3, 3),
                  "GB_s": round(src.numel() / el / 1e9, 2)})
            del dst
    from agent_tpu_amd.utils.synthetic import write_csv

    csv = f"/tmp/atpu_cold_{a.rows}.csv"
    if not os.path.exists(csv):
        write_csv(csv, 2 * a.rows, 150, seed=5)
    os.environ.setdefault("TASKS", "map_classify")
    from ops import get_op

    op = get_op("map_classify")
    # first load of the process (imports, code objects, allocator), then LRU misses in a warm
    # process: MODEL_LRU_SIZE=1 evicts each model when the next one loads, so the last entry
    # (the first model again) is a miss too
    os.environ["MODEL_LRU_SIZE"] = "1"
    models = [m for m in a.classify.split(",") if m]
    for i, model in enumerate(models + models[:1]):
        rec = {"what": "classify_cold_load", "model": model, "process": "fresh" if i == 0 else "warm (LRU miss)"}
        for phase in ("cold", "warm"):
            t0 = time.perf_counter()
            out = op({"source_uri": csv, "start_row": 0, "shard_size": a.rows, "text_column": "text", "topk": 2,
                      "output": "summary", "model_path": model})
            torch.cuda.synchronize(dev)
            rec[f"{phase}_job_ms"] = ms(t0)
            tm = (out.get("timing_ms") or {}) if isinstance(out, dict) else {}
            if phase == "cold":
                rec["cold_load"] = tm.get("cold_load")
                rec["load_ms"] = tm.get("load_ms")
            assert isinstance(out, dict) and out.get("ok", True), out
        rec["miss_overhead_ms"] = round(rec["cold_job_ms"] - rec["warm_job_ms"], 2)
        emit(rec)
    for model in [m for m in a.summarize.split(",") if m]:
        from agent_tpu_amd.runtime.summarize import SummarizeEngine, build_model

        t0 = time.perf_counter()
        m, pack = build_model(model, device=dev, seed=0)
        torch.cuda.synchronize(dev)
        w = ms(t0)
        eng = SummarizeEngine(m, max_source_len=1024)
        torch.cuda.synchronize(dev)
        emit({"what": "summarize_cold_load", "model": model, "weights_ms": w, "total_ms": ms(t0),
              "weight_bytes": int(pack.nbytes)})
        del eng, m, pack
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
