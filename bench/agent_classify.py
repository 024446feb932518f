#!/usr/bin/env python3
"""Whole-agent classify throughput on one GPU: the real ``app.py`` leases ``map_classify``
CSV-shard jobs from a local mock controller and posts their per-row top-k results back.

Unlike ``bench.py`` (the engine alone) the clock here covers everything a deployed agent
does per job: lease over HTTP, the native CSV index, pinned staging, the BERT pipeline on
the GPU, building the reference-format JSON result (one dict per row, or the
``output: "summary"`` histogram) and posting it. It runs from the first lease request to
the last result; the model load (first job) is excluded by a warm-up job.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from tests.integration.mock_controller import MockController  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=16)
    ap.add_argument("--shard", type=int, default=16384, help="CSV rows per job")
    ap.add_argument("--output", default="rows", choices=["rows", "columns", "summary"])
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--form", default="csv", choices=["csv", "input"],
                    help="csv: CSV-shard jobs; input: the reference job shape, one pre-tokenized row per job")
    ap.add_argument("--max-tasks", type=int, default=1, help="MAX_TASKS (input form: jobs per lease, batched)")
    ap.add_argument("--batch", default="1", help="LEASE_BATCH")
    ap.add_argument("--inflight-depth", default="1",
                    help="INFLIGHT_DEPTH of the agent: 1 = the serial loop, N or auto = in-flight (many leases held)")
    ap.add_argument("--dp", type=int, default=1,
                    help="agent ranks (torch.distributed.run, one process per GPU; rank 0 leases)")
    ap.add_argument("--controller", default="fast", choices=["fast", "mock"],
                    help="input form: the asyncio stand-in (bench/fast_controller.py) or the test mock "
                         "(ThreadingHTTPServer, itself the ceiling at ~6-7k results/s)")
    ap.add_argument("--dp-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks on fewer GPUs (ranks share a card)")
    a = ap.parse_args()
    if a.form == "input":
        return input_form(a)
    from agent_tpu_amd.utils.synthetic import write_csv

    rows = (a.jobs + 1) * a.shard
    csv_path = f"/tmp/atpu_agent_bench_{rows}.csv"
    if not os.path.exists(csv_path):
        write_csv(csv_path, rows, 150, seed=77)
    ctl = MockController().start()

    def job(i):
        return {"id": f"j{i}", "op": "map_classify",
                "payload": {"source_uri": csv_path, "start_row": i * a.shard, "shard_size": a.shard,
                            "text_column": "text", "topk": 2, "output": a.output, "dataset_id": "bench"}}

    ctl.lease(job(0), lease_id="Lwarm")  # model load + graph capture
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="map_classify", IDLE_SLEEP_SEC="0.01", MAX_TASKS="1",
               GPU_MODEL_PATH=a.model, PYTHONUNBUFFERED="1", ATPU_DP_BACKEND=a.dp_backend)
    cmd = [sys.executable, "app.py"]
    if a.dp > 1:
        from agent_tpu_amd.parallel.launch import torchrun_cmd

        cmd = torchrun_cmd("app.py", [], a.dp)
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        ok = ctl.wait(lambda c: len(c.results) >= 1, 600)
        for i in range(1, a.jobs + 1):
            ctl.lease(job(i), lease_id=f"L{i}")
        t0 = time.perf_counter()
        ok = ok and ctl.wait(lambda c: len(c.results) >= a.jobs + 1, 1200)
        el = time.perf_counter() - t0
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=120)
        ctl.stop()
    bad = [r for r in ctl.results if r.get("status") != "succeeded"]
    if not ok or bad:
        print(json.dumps({"error": "timeout" if not ok else "failed jobs", "results": len(ctl.results),
                          "first_bad": bad[:1]}, default=str)[:2000])
        return 1
    prof = (ctl.lease_requests[0].get("worker_profile") or {}) if ctl.lease_requests else {}
    rank_table = ((prof.get("gpu") or {}).get("health") or {}).get("ranks")
    first = ctl.results[0]["result"]  # the warm-up job: it paid the model's cold load
    ftm = first.get("timing_ms") or {}
    first_job = {"elapsed_ms": first.get("elapsed_ms"), "load_ms": ftm.get("load_ms"), "cold_load": ftm.get("cold_load")}
    res = [r["result"] for r in ctl.results[1:]]
    n = sum(int(r["row_count"]) for r in res)
    engine_rps = sorted(float(r["rows_per_sec"]) for r in res)[len(res) // 2]
    keys = sorted({k for r in res for k in (r.get("timing_ms") or {})})
    timing = {k: round(sorted(float((r.get("timing_ms") or {}).get(k, 0.0)) for r in res)[len(res) // 2], 2)
              for k in keys}
    op_ms = round(sorted(float(r["elapsed_ms"]) for r in res)[len(res) // 2], 2)
    print(json.dumps({"metric": f"classified rows/sec end to end through the agent ({a.model}, 1 GPU)",
                      "value": round(n / el, 1), "unit": "rows/s", "higher_is_better": True,
                      "config": {"jobs": a.jobs, "rows_per_job": a.shard, "output": a.output,
                                 "dp_ranks": a.dp, "dp_backend": a.dp_backend if a.dp > 1 else None,
                                 "median_op_rows_per_sec": round(engine_rps, 1),
                                 "median_op_elapsed_ms": op_ms, "median_op_timing_ms": timing,
                                 "first_job_cold_model": first_job, "rank_table": rank_table,
                                 "transport": "HTTP/1.1 keep-alive, loopback mock controller",
                                 "data": "synthetic CSV rows, random-init weights"}}), flush=True)
    return 0


def input_form(a) -> int:
    """Reference-shaped jobs (``{"input": [128 token ids]}``, one row each; ref
    ``ops/map_classify_tpu.py:52-75``), MAX_TASKS per lease, batched on the GPU."""
    import numpy as np

    rng = np.random.default_rng(3)
    S = 128

    def ids(i):
        n = int(rng.integers(16, S - 2))
        return [101] + [int(x) for x in rng.integers(1000, 30000, n)] + [102] + [0] * (S - n - 2)

    if a.controller == "fast":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from fast_controller import FastController

        ctl = FastController().start()
        count = lambda c: c.n_results()  # noqa: E731
    else:
        ctl = MockController().start()
        count = lambda c: len(c.results)  # noqa: E731

    def job(i):
        return {"id": f"j{i}", "op": "map_classify", "job_epoch": i,
                "payload": {"input": ids(i), "topk": 2, "model_path": a.model}}

    ctl.lease(*[job(-1 - i) for i in range(a.max_tasks)], lease_id="Lwarm")
    nwarm = a.max_tasks
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="map_classify", IDLE_SLEEP_SEC="0.01",
               MAX_TASKS=str(a.max_tasks), LEASE_BATCH=a.batch, PYTHONUNBUFFERED="1",
               INFLIGHT_DEPTH=str(a.inflight_depth))
    p = subprocess.Popen([sys.executable, "app.py"], cwd=REPO, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    try:
        ok = ctl.wait(lambda c: count(c) >= nwarm, 600)
        for b0 in range(0, a.jobs, a.max_tasks):
            ctl.lease(*[job(i) for i in range(b0, min(a.jobs, b0 + a.max_tasks))], lease_id=f"L{b0}")
        t0 = time.perf_counter()
        ok = ok and ctl.wait(lambda c: count(c) >= nwarm + a.jobs, 1200)
        el = time.perf_counter() - t0
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=120)
        ctl.stop()
    res = ctl.results[nwarm:]
    bad = [r for r in res if r.get("status") != "succeeded" or "fallback" in (r.get("result") or {})]
    if not ok or bad:
        print(json.dumps({"error": "timeout" if not ok else "failed jobs", "results": len(res),
                          "first_bad": bad[:1]}, default=str)[:2000])
        return 1
    lat = _latencies(ctl, res, nwarm, a.max_tasks)
    print(json.dumps({"metric": f"classified rows/sec end to end through the agent, 1-row input jobs ({a.model}, 1 GPU)",
                      "value": round(a.jobs / el, 1), "unit": "rows/s", "higher_is_better": True,
                      "config": {"jobs": a.jobs, "max_tasks": a.max_tasks, "lease_batch": a.batch, "seq_len": S,
                                 "jobs_per_lease": a.max_tasks, "leases_per_sec": round(a.jobs / a.max_tasks / el, 1),
                                 "result_keys": sorted(res[0]["result"]),
                                 "inflight_depth": a.inflight_depth, "job_latency_ms": lat,
                                 "controller": a.controller,
                                 "transport": "HTTP/1.1 keep-alive, loopback mock controller",
                                 "data": "synthetic token ids, random-init weights"}}), flush=True)
    return 0


def _latencies(ctl, res, nwarm: int, per_lease: int):
    """Per-job latency (lease answered -> result received at the controller), ms: p50 / p99 / max.
    Timed job i rode lease 1 + i // per_lease (lease 0 is the warm-up lease)."""
    lt = list(getattr(ctl, "lease_t", []) or [])
    rt = list(getattr(ctl, "result_t", []) or [])
    if lt and rt:
        out = []
        for k, r in enumerate(res):
            i = int(r["job_id"][1:])
            li = 1 + i // per_lease
            if li < len(lt) and nwarm + k < len(rt):
                out.append((rt[nwarm + k] - lt[li]) * 1e3)
    else:  # the test mock: wall-clock stamps by id
        out = [(ctl.result_times[r["job_id"]] - ctl.lease_times[f"L{(int(r['job_id'][1:]) // per_lease) * per_lease}"]) * 1e3
               for r in res if r["job_id"] in ctl.result_times]
    if not out:
        return None
    out.sort()
    return {"p50": round(out[len(out) // 2], 1), "p99": round(out[min(len(out) - 1, int(0.99 * len(out)))], 1),
            "max": round(out[-1], 1)}


if __name__ == "__main__":
    sys.exit(main())
