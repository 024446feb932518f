#!/usr/bin/env python3
"""Host CSV ingest rate for N concurrent DP ranks.

At DP=8 each rank's HostStager extracts its own row range of the shard through the
native CSV index (``CsvTable.extract_column``: byte-offset row index, field slicing,
packed UTF-8 + offsets). This runs N independent processes, one per simulated rank,
each extracting 1024-row batches of its contiguous range into pageable buffers (the
production stager writes pinned ones; same parsing work), and reports the aggregate
rows/s. The engine consumes ~49k rows/s per MI355X (BERT-base, S=128), so the host
must sustain N x 49k.

  python bench/ingest_scaling.py --procs 1,2,4,8 --rows 400000
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _rank(path: str, start: int, n: int, batch: int, threads: int, q) -> None:
    from agent_tpu_amd._native import native

    t = native().CsvTable(path)
    col = t.column_index("text")
    t0 = time.perf_counter()
    done, nbytes = 0, 0
    for b in range(start, start + n, batch):
        m = min(batch, start + n - b)
        text, offs = t.extract_column(b, m, col, 4096, threads)
        done += m
        nbytes += int(text.nbytes)
    q.put((done, nbytes, time.perf_counter() - t0))


def run(path: str, rows: int, procs: int, batch: int, threads: int):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    per = rows // procs
    ps = [ctx.Process(target=_rank, args=(path, p * per, per, batch, threads, q)) for p in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    wall = max(r[2] for r in res)
    done = sum(r[0] for r in res)
    return {"procs": procs, "rows": done, "max_rank_s": round(wall, 3), "rows_per_sec": round(done / wall, 1),
            "MB_per_sec": round(sum(r[1] for r in res) / wall / 1e6, 1)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,2,4,8")
    ap.add_argument("--rows", type=int, default=400_000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=1, help="extraction threads per rank")
    ap.add_argument("--words", type=int, default=150)
    a = ap.parse_args()
    from agent_tpu_amd.utils.synthetic import write_csv

    path = f"/tmp/atpu_ingest_{a.rows}_{a.words}.csv"
    if not os.path.exists(path):
        write_csv(path, a.rows, a.words, seed=11)
    from agent_tpu_amd._native import native

    native().CsvTable(path)  # build (and cache) the row index once, outside the timing
    out = [run(path, a.rows, int(p), a.batch, a.threads) for p in a.procs.split(",")]
    print(json.dumps({"metric": "host CSV ingest rows/sec, N concurrent rank stagers (native CSV index)",
                      "unit": "rows/s", "cpus": os.cpu_count(), "words_per_row": a.words,
                      "bytes_per_row": round(os.path.getsize(path) / a.rows, 1), "batch_rows": a.batch,
                      "threads_per_rank": a.threads, "points": out,
                      "engine_rate_per_gpu": 49000}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
