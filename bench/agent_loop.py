#!/usr/bin/env python3
"""Agent control-plane throughput: echo jobs/s end to end against a local mock
controller (BASELINE config 1; SURVEY.md §6 B1: reference ~386 jobs/s on an
8-vCPU VM over loopback, one TCP connection per request, one task per lease).

Runs the real ``app.py`` as a subprocess; the controller serves ``--jobs``
echo tasks in leases of ``--max-tasks`` and the clock runs from the first lease
to the last result.
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

BASELINE_JOBS_PER_SEC = 386.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=5000)
    ap.add_argument("--max-tasks", type=int, default=1)
    ap.add_argument("--controller", default="mock", choices=["mock", "fast"],
                    help="fast: the asyncio stand-in (bench/fast_controller.py) instead of the test mock")
    a = ap.parse_args()
    if a.controller == "fast":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from fast_controller import FastController

        ctl = FastController().start()
    else:
        ctl = MockController().start()
    k = max(1, a.max_tasks)
    for i in range(0, a.jobs, k):
        ctl.lease(*[{"id": f"j{j}", "op": "echo", "payload": {"i": j}} for j in range(i, min(a.jobs, i + k))],
                  lease_id=f"L{i}")
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="echo", IDLE_SLEEP_SEC="0.01", MAX_TASKS=str(k),
               GPU_DISABLED="1", PYTHONUNBUFFERED="1")
    p = subprocess.Popen([sys.executable, "app.py"], cwd=REPO, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    try:
        ok = ctl.wait(lambda c: len(c.lease_requests) >= 1, 120)
        t0 = time.perf_counter()
        count = (lambda c: c.n_results()) if a.controller == "fast" else (lambda c: len(c.results))
        ok = ok and ctl.wait(lambda c: count(c) >= a.jobs, 600)
        el = time.perf_counter() - t0
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=60)
        ctl.stop()
    if not ok:
        print(json.dumps({"error": "timeout", "results": len(ctl.results)}))
        return 1
    v = a.jobs / el
    print(json.dumps({"metric": "echo jobs/sec end to end (agent loop vs mock controller)", "value": round(v, 1),
                      "unit": "jobs/s", "higher_is_better": True, "vs_baseline": round(v / BASELINE_JOBS_PER_SEC, 2),
                      "config": {"jobs": a.jobs, "max_tasks": k, "controller": a.controller,
                                 "transport": "HTTP/1.1 keep-alive, loopback"}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
