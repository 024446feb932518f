#!/usr/bin/env python3
"""Whole-agent summarize throughput on reference-shaped jobs: ONE document per job.

The reference leases one ``map_summarize`` ``{"text": ...}`` job per task and decodes it
at batch 1 (ref ``app.py:191,286-287``, ``ops/map_summarize.py:39-59``). Here the real
``app.py`` leases ``MAX_TASKS`` such jobs at once from a local mock controller and runs
them as one beam-search batch (app.py ``run_tasks`` -> ``ops.map_summarize.handle_batch``),
posting one result per job. The clock runs from the first lease of the timed jobs to the
last result; a warm-up lease (model build, graph capture) is excluded.

  python bench/agent_summarize.py --jobs 512 --max-tasks 256 [--model bart-large-cnn]
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
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--jobs", type=int, default=512)
    ap.add_argument("--max-tasks", type=int, default=256)
    ap.add_argument("--src-len", type=int, default=1024)
    ap.add_argument("--batch", default="1", help="LEASE_BATCH (0 = job by job, the reference's shape)")
    ap.add_argument("--inflight-depth", default="1",
                    help="INFLIGHT_DEPTH of the agent: 1 = the serial loop, N or auto = in-flight (many leases held; "
                         "documents join running searches at decode-step boundaries)")
    a = ap.parse_args()
    from agent_tpu_amd.utils.synthetic import make_text_rows

    docs = make_text_rows(a.jobs + a.max_tasks, words_per_row=int(a.src_len * 0.8), seed=5)
    ctl = MockController().start()

    def job(i):
        return {"id": f"j{i}", "op": "map_summarize", "job_epoch": i, "payload": {"text": docs[i]}}

    warm = [job(a.jobs + i) for i in range(a.max_tasks)]
    ctl.lease(*warm, lease_id="Lwarm")
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="map_summarize", IDLE_SLEEP_SEC="0.01",
               MAX_TASKS=str(a.max_tasks), LEASE_BATCH=a.batch, SUMMARIZE_MODEL=a.model,
               SUMMARIZE_MAX_SOURCE_TOKENS=str(a.src_len), PYTHONUNBUFFERED="1",
               INFLIGHT_DEPTH=str(a.inflight_depth))
    p = subprocess.Popen([sys.executable, "app.py"], cwd=REPO, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    try:
        ok = ctl.wait(lambda c: len(c.results) >= len(warm), 900)
        for b0 in range(0, a.jobs, a.max_tasks):
            ctl.lease(*[job(i) for i in range(b0, min(a.jobs, b0 + a.max_tasks))], lease_id=f"L{b0}")
        t0 = time.perf_counter()
        ok = ok and ctl.wait(lambda c: len(c.results) >= len(warm) + a.jobs, 1800)
        el = time.perf_counter() - t0
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=120)
        ctl.stop()
    res = ctl.results[len(warm):]
    bad = [r for r in res if r.get("status") != "succeeded" or not (r.get("result") or {}).get("ok")]
    if not ok or bad:
        print(json.dumps({"error": "timeout" if not ok else "failed jobs", "results": len(res),
                          "first_bad": bad[:1]}, default=str)[:2000])
        return 1
    epochs_ok = all(r["job_epoch"] == int(r["job_id"][1:]) for r in res)
    per_job_ms = sorted(float(r["result"]["elapsed_ms"]) for r in res)
    lat = sorted((ctl.result_times[r["job_id"]] - ctl.lease_times[f"L{(int(r['job_id'][1:]) // a.max_tasks) * a.max_tasks}"])
                 * 1e3 for r in res)
    lat_ms = {"p50": round(lat[len(lat) // 2], 1), "p99": round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 1),
              "max": round(lat[-1], 1)}
    print(json.dumps({"metric": f"summarized docs/sec end to end through the agent, 1-doc jobs ({a.model}, 1 GPU)",
                      "value": round(a.jobs / el, 2), "unit": "docs/s", "higher_is_better": True,
                      "config": {"jobs": a.jobs, "max_tasks": a.max_tasks, "lease_batch": a.batch,
                                 "src_len": a.src_len, "num_beams": 4, "max_length": 130, "min_length": 30,
                                 "batched_docs": res[0]["result"].get("batched_docs", 1),
                                 "median_job_elapsed_ms": round(per_job_ms[len(per_job_ms) // 2], 1),
                                 "inflight_depth": a.inflight_depth, "job_latency_ms": lat_ms,
                                 "searches_batched_docs_median": sorted(r["result"].get("batched_docs", 1)
                                                                         for r in res)[len(res) // 2],
                                 "epochs_passed_through": epochs_ok,
                                 "transport": "HTTP/1.1 keep-alive, loopback mock controller",
                                 "data": "synthetic text documents, random-init weights"}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
