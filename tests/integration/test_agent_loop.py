"""Agent loop against the mock controller: wire protocol, multi-task leases,
bad tasks, result retry policy, signals and exit codes.

The real ``app.py`` runs as a subprocess with env overrides (CPU only).
"""
import os
import signal
import subprocess
import sys
import time

import pytest

from .mock_controller import MockController

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.fixture
def ctl():
    c = MockController().start()
    yield c
    c.stop()


def start_agent(ctl, tasks="echo,risk_accumulate,read_csv_shard,map_tokenize", **env):
    e = dict(os.environ)
    e.update({"CONTROLLER_URL": ctl.url, "TASKS": tasks, "IDLE_SLEEP_SEC": "0.02", "ERROR_BACKOFF_SEC": "0.05",
              "ERROR_LOG_EVERY_SEC": "0", "AGENT_NAME": "test-agent", "AGENT_LABELS": "zone=a,gpu,x=1=2",
              "PYTHONUNBUFFERED": "1", "GPU_DISABLED": "1", "HIP_VISIBLE_DEVICES": ""})
    e.update({k: str(v) for k, v in env.items()})
    return subprocess.Popen([sys.executable, "app.py"], cwd=REPO, env=e, stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)


def stop_agent(p, sig=signal.SIGTERM, timeout=30):
    p.send_signal(sig)
    out, _ = p.communicate(timeout=timeout)
    return p.returncode, out


def by_job(ctl):
    return {r["job_id"]: r for r in ctl.results}


def test_protocol_and_ops(ctl, tmp_path):
    csv = tmp_path / "s.csv"
    csv.write_text("id,text,risk\n1,a,0.5\n2,b,1.5\n3,c,2.5\n")
    ctl.lease({"id": "j1", "op": "echo", "payload": {"x": 1}, "job_epoch": 7})
    ctl.lease({"job_id": "j2", "op": "risk_accumulate", "payload": {"values": [1, "2", 3.5]}, "job_epoch": 1})
    ctl.lease({"id": "j3", "op": "read_csv_shard", "payload": {"source_uri": str(csv), "start_row": 1,
                                                              "shard_size": 5}})
    ctl.lease({"id": "j4", "op": "map_tokenize", "payload": {"text": "abcdef", "chunk_size": 4}})
    ctl.lease({"id": "j5", "op": "risk_accumulate", "payload": {"values": "bad"}})
    ctl.lease({"id": "j6", "op": "nope", "payload": {}})
    ctl.lease({"op": "echo", "payload": {}})  # no id: skipped, never resulted
    ctl.lease({"id": "j8", "op": "echo", "payload": []})  # payload [] is falsy -> {} like the reference
    p = start_agent(ctl)
    try:
        assert ctl.wait(lambda c: len(c.results) >= 7, 90), ctl.results
        n = len(ctl.lease_requests)
        assert ctl.wait(lambda c: len(c.lease_requests) > n, 30)  # next lease carries updated metrics
    finally:
        code, out = stop_agent(p)
    assert code == 0, out
    r = by_job(ctl)
    assert r["j1"] == {"lease_id": "L1", "job_id": "j1", "job_epoch": 7, "status": "succeeded",
                       "result": {"ok": True, "echo": {"x": 1}}, "error": None}
    assert r["j2"]["status"] == "succeeded" and r["j2"]["job_epoch"] == 1
    assert r["j2"]["result"]["count"] == 3 and r["j2"]["result"]["sum"] == 6.5
    rows = r["j3"]["result"]["rows"]
    assert r["j3"]["status"] == "succeeded" and [x["id"] for x in rows] == ["2", "3"]
    assert r["j4"]["result"]["tokens"] == ["abcd", "ef"]
    assert r["j5"]["status"] == "failed" and r["j5"]["result"] is None
    assert r["j5"]["error"]["type"] == "ValueError" and r["j5"]["error"]["message"] == "payload.values must be a list"
    assert "Traceback" in r["j5"]["error"]["trace"]
    assert r["j6"]["status"] == "failed" and "Unknown op 'nope'" in r["j6"]["error"]["message"]
    assert r["j8"]["result"] == {"ok": True, "echo": {}}
    assert len(ctl.results) == 7  # the id-less task is never resulted
    assert "bad task" in out
    req = ctl.lease_requests[0]
    assert set(req) == {"agent", "capabilities", "max_tasks", "timeout_ms", "labels", "worker_profile", "metrics"}
    assert req["agent"] == "test-agent" and req["max_tasks"] == 1 and req["timeout_ms"] == 3000
    assert req["capabilities"] == {"ops": ["echo", "risk_accumulate", "read_csv_shard", "map_tokenize"]}
    assert req["labels"] == {"zone": "a", "gpu": True, "x": "1=2"}
    prof = req["worker_profile"]
    assert {"cpu", "gpu", "workers", "tier", "limits"} <= set(prof)
    assert prof["limits"] == {"max_payload_bytes": 262144, "max_tokens": 2048}
    assert {"jobs_completed", "jobs_failed", "rows_per_sec"} <= set(req["metrics"])
    later = ctl.lease_requests[-1]["metrics"]
    assert later["jobs_completed"] >= 5 and later["jobs_failed"] >= 2


def test_multi_task_lease_runs_every_task(ctl):
    ctl.lease(*[{"id": f"m{i}", "op": "echo", "payload": {"i": i}} for i in range(3)], lease_id="LM")
    p = start_agent(ctl, MAX_TASKS=3)
    try:
        assert ctl.wait(lambda c: len(c.results) >= 3, 60)
    finally:
        code, _ = stop_agent(p)
    assert code == 0
    assert [r["job_id"] for r in ctl.results] == ["m0", "m1", "m2"]
    assert all(r["lease_id"] == "LM" for r in ctl.results)
    assert ctl.lease_requests[0]["max_tasks"] == 3


def test_result_retry_policy(ctl):
    ctl.result_codes = {"stale": [409], "flaky": [500, 503], "dead": [500, 500, 500, 500]}
    for jid in ("stale", "flaky", "dead", "after"):
        ctl.lease({"id": jid, "op": "echo", "payload": {}})
    p = start_agent(ctl, RESULT_RETRIES=2)
    try:
        assert ctl.wait(lambda c: "after" in c.result_attempts, 60)
    finally:
        code, out = stop_agent(p)
    assert code == 0
    assert ctl.result_attempts["stale"] == 1  # 4xx is final (stale epoch)
    assert ctl.result_attempts["flaky"] == 3 and "flaky" in by_job(ctl)
    assert ctl.result_attempts["dead"] == 3 and "dead" not in by_job(ctl)
    assert "post result error" in out


def test_lease_errors_back_off_and_recover(ctl):
    ctl.lease(status=500, body={"error": "boom"})
    ctl.lease(status=200, body={"no_lease_id": True})
    ctl.lease(status=200, body=["not", "a", "dict"])
    ctl.lease({"id": "ok1", "op": "echo", "payload": {}})
    p = start_agent(ctl)
    try:
        assert ctl.wait(lambda c: len(c.results) >= 1, 60)
    finally:
        code, out = stop_agent(p)
    assert code == 0 and by_job(ctl)["ok1"]["status"] == "succeeded"
    assert "lease error" in out


def test_sigint_and_idle(ctl):
    p = start_agent(ctl)
    assert ctl.wait(lambda c: len(c.lease_requests) >= 3, 60)  # 204s -> idle polling
    code, out = stop_agent(p, signal.SIGINT)
    assert code == 0 and "stopped" in out


def test_no_tasks_exits_2(ctl):
    p = start_agent(ctl, tasks="")
    out, _ = p.communicate(timeout=60)
    assert p.returncode == 2 and "no TASKS" in out
    assert not ctl.lease_requests


def test_unavailable_op_not_advertised(ctl):
    p = start_agent(ctl, tasks="echo,definitely_not_an_op")
    try:
        assert ctl.wait(lambda c: len(c.lease_requests) >= 1, 60)
    finally:
        code, out = stop_agent(p)
    assert ctl.lease_requests[0]["capabilities"]["ops"] == ["echo"]
    assert "op unavailable: definitely_not_an_op" in out


def test_async_result_poster_keeps_every_result(ctl):
    """RESULT_POST_ASYNC=1: results go out from a background thread, in order, each with
    its job_epoch, and SIGTERM flushes the queue before exit."""
    for i in range(12):
        ctl.lease({"id": f"a{i}", "op": "echo", "payload": {"i": i}, "job_epoch": i})
    ctl.result_codes["a3"] = [500, 200]  # retried by the poster, still delivered
    p = start_agent(ctl, tasks="echo", RESULT_POST_ASYNC="1")
    try:
        assert ctl.wait(lambda c: len(c.results) >= 12, 60), ctl.results
    finally:
        code, out = stop_agent(p)
    assert code == 0, out
    got = [(r["job_id"], r["job_epoch"], r["result"]["echo"]["i"]) for r in ctl.results]
    # every result exactly once with its epoch, FIFO except the retried one (with RESULT_PIPELINE
    # the results queued behind it were already on the wire when its 500 came back)
    assert sorted(got) == sorted((f"a{i}", i, i) for i in range(12))
    assert [g for g in got if g[0] != "a3"] == [(f"a{i}", i, i) for i in range(12) if i != 3]
    assert ctl.result_attempts["a3"] == 2


def _order(ctl):
    return [e for e in ctl.events if e != ("lease", None)]


def test_lease_prefetch_and_async_post_overlap_jobs(ctl):
    """with the defaults the next lease is taken while the current job's
    result is still being posted (a slow controller: 0.3 s per result answer), results stay
    in FIFO order with their epochs; LEASE_PREFETCH=0 RESULT_POST_ASYNC=0 is the reference's
    strict lease -> execute -> post order."""
    ctl.result_delay = 0.3
    for i in range(3):
        ctl.lease({"id": f"p{i}", "op": "echo", "payload": {"i": i}, "job_epoch": 10 + i}, lease_id=f"P{i}")
    p = start_agent(ctl, tasks="echo")
    try:
        assert ctl.wait(lambda c: len(c.results) >= 3, 60), ctl.results
    finally:
        code, out = stop_agent(p)
    assert code == 0, out
    ev = _order(ctl)
    assert ev.index(("lease", "P1")) < ev.index(("result", "p0")), ev  # leased ahead, posted behind
    assert [(r["job_id"], r["job_epoch"], r["lease_id"]) for r in ctl.results] == \
        [(f"p{i}", 10 + i, f"P{i}") for i in range(3)]


def test_serial_order_when_disabled(ctl):
    ctl.result_delay = 0.1
    for i in range(3):
        ctl.lease({"id": f"s{i}", "op": "echo", "payload": {}}, lease_id=f"S{i}")
    p = start_agent(ctl, tasks="echo", LEASE_PREFETCH="0", RESULT_POST_ASYNC="0")
    try:
        assert ctl.wait(lambda c: len(c.results) >= 3, 60), ctl.results
    finally:
        code, out = stop_agent(p)
    assert code == 0, out
    assert _order(ctl)[:6] == [("lease", "S0"), ("result", "s0"), ("lease", "S1"), ("result", "s1"),
                               ("lease", "S2"), ("result", "s2")]


_SHUTDOWN_DRIVER = r'''
import os, signal, threading, time
import app
app._running = True
signal.signal(signal.SIGTERM, app._on_signal)
agent = app.Agent()
def slow(payload):
    # SIGTERM arrives while this job runs, once the next lease has been taken ahead
    def kick():
        while agent._leaser is None or not agent._leaser.pending():
            time.sleep(0.01)
        os.kill(os.getpid(), signal.SIGTERM)
    threading.Thread(target=kick, daemon=True).start()
    time.sleep(1.0)
    return {"ok": True}
agent.handlers["slow"] = slow
agent.loop()
agent.flush_results()
print("exited")
'''


def _run_shutdown_driver(ctl, **env):
    e = dict(os.environ)
    e.update({"CONTROLLER_URL": ctl.url, "TASKS": "echo", "GPU_DISABLED": "1", "HIP_VISIBLE_DEVICES": "",
              "PYTHONUNBUFFERED": "1", "IDLE_SLEEP_SEC": "0.02"})
    e.update(env)
    r = subprocess.run([sys.executable, "-c", _SHUTDOWN_DRIVER], cwd=REPO, env=e, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "exited" in r.stdout, r.stdout + r.stderr
    return r.stdout


def test_sigterm_does_not_start_the_prefetched_lease(ctl):
    """VERDICT r5 #7 (ref app.py:239-242,257): after SIGTERM only the running batch finishes.
    A lease taken ahead is not started; by default nothing is posted for it (the controller
    re-leases it when the lease TTL runs out)."""
    ctl.lease({"id": "t0", "op": "slow", "payload": {}}, lease_id="T0")
    ctl.lease({"id": "t1", "op": "echo", "payload": {}}, lease_id="T1")
    out = _run_shutdown_driver(ctl)
    assert [r["job_id"] for r in ctl.results] == ["t0"]
    assert ("lease", "T1") in ctl.events
    assert "leased ahead not started; left to the lease TTL (lease T1)" in out


def test_sigterm_fails_the_prefetched_lease_when_asked(ctl):
    ctl.lease({"id": "u0", "op": "slow", "payload": {}}, lease_id="U0")
    ctl.lease({"id": "u1", "op": "echo", "payload": {}, "job_epoch": 4}, lease_id="U1")
    _run_shutdown_driver(ctl, SHUTDOWN_AHEAD="fail")
    r = by_job(ctl)
    assert r["u0"]["status"] == "succeeded"
    assert r["u1"]["status"] == "failed" and r["u1"]["error"]["type"] == "Shutdown"
    assert r["u1"]["lease_id"] == "U1" and r["u1"]["job_epoch"] == 4


_DRIVER = r'''
import json, sys, threading, time
import app
agent = app.Agent()
t_done = {}
def slow(payload):
    time.sleep(float(payload["sec"]))
    t_done["slow"] = time.time()
    return {"ok": True}
agent.handlers["slow"] = slow
agent.run_tasks("L9", [{"id": "e0", "op": "echo", "payload": {}}, {"id": "s0", "op": "slow", "payload": {"sec": 1.5}}])
agent.flush_results()
print(json.dumps(t_done))
'''


def test_short_result_is_not_held_behind_a_slow_job(ctl):
    """in a lease [echo, slow job] the echo result reaches the controller before
    the slow job ends (grouped posts never wait behind a job that may be long)."""
    e = dict(os.environ)
    e.update({"CONTROLLER_URL": ctl.url, "TASKS": "echo", "GPU_DISABLED": "1", "HIP_VISIBLE_DEVICES": "",
              "PYTHONUNBUFFERED": "1"})
    r = subprocess.run([sys.executable, "-c", _DRIVER], cwd=REPO, env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    import json

    slow_end = json.loads(r.stdout.strip().splitlines()[-1])["slow"]
    arrived = ctl.result_times
    assert arrived["e0"] < slow_end - 1.0, (arrived, slow_end)
    assert "s0" in arrived


def test_inflight_echo_jobs_hold_many_leases(ctl):
    """INFLIGHT_DEPTH: one job per lease, leases requested pipelined while earlier jobs run;
    every job resulted once with its lease and epoch."""
    for i in range(40):
        ctl.lease({"id": f"f{i}", "op": "echo", "payload": {"i": i}, "job_epoch": i}, lease_id=f"F{i}")
    p = start_agent(ctl, tasks="echo", MAX_TASKS=1, INFLIGHT_DEPTH=16)
    try:
        assert ctl.wait(lambda c: len(c.results) >= 40, 60), ctl.results
    finally:
        code, out = stop_agent(p)
    assert code == 0, out
    assert "in-flight mode: up to 16 leased jobs held" in out
    got = sorted((r["job_id"], r["lease_id"], r["job_epoch"], r["result"]["echo"]["i"]) for r in ctl.results)
    assert got == sorted((f"f{i}", f"F{i}", i, i) for i in range(40))
    assert all(r["max_tasks"] == 1 for r in ctl.lease_requests)


def test_inflight_is_off_for_a_cpu_agent_by_default(ctl):
    ctl.lease({"id": "g0", "op": "echo", "payload": {}}, lease_id="G0")
    p = start_agent(ctl, tasks="echo")
    try:
        assert ctl.wait(lambda c: len(c.results) >= 1, 60)
    finally:
        code, out = stop_agent(p)
    assert code == 0 and "in-flight mode" not in out
