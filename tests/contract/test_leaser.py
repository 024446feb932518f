"""app.Leaser (LEASE_PREFETCH): the next lease is taken by a helper thread only while a
batch has been running for LEASE_PREFETCH_AFTER_MS; short batches keep the serial order."""
import threading
import time

import pytest


class FakeCtl:
    log = []
    queue = []
    lock = threading.Lock()

    def __init__(self, *a, **k):
        pass

    def lease(self, caps, profile):
        with FakeCtl.lock:
            FakeCtl.log.append((threading.current_thread().name, time.monotonic()))
            return FakeCtl.queue.pop(0) if FakeCtl.queue else None


class FakeAgent:
    caps = ["echo"]
    profile = {}
    ctl = FakeCtl()


@pytest.fixture
def leaser(monkeypatch):
    import app

    monkeypatch.setattr(app, "Controller", FakeCtl)
    monkeypatch.setattr(app, "IDLE_SLEEP_SEC", 0.0)
    monkeypatch.setenv("LEASE_PREFETCH_AFTER_MS", "5")
    FakeCtl.log, FakeCtl.queue = [], [("L%d" % i, [{"id": str(i)}]) for i in range(4)]
    lz = app.Leaser(FakeAgent())
    yield lz
    lz.stop()


def test_long_batch_gets_its_next_lease_ahead(leaser):
    first = leaser.next()
    assert first[0] == "L0" and FakeCtl.log[-1][0] == "MainThread"
    leaser.started()
    time.sleep(0.1)  # a long batch: the helper leases L1 after 5 ms
    assert leaser.pending() == [("L1", [{"id": "1"}])]
    assert [n for n, _ in FakeCtl.log] == ["MainThread", "atpu-leaser"]
    leaser.finished()
    assert leaser.next()[0] == "L1" and len(FakeCtl.log) == 2  # no new request
    leaser.started()
    time.sleep(0.1)
    leaser.finished()
    assert leaser.pending() == [("L2", [{"id": "2"}])]  # one ahead per batch, never more


def test_lease_ahead_waits_for_the_expected_end_of_long_batches(leaser, monkeypatch):
    """the ahead lease is taken ~LEASE_PREFETCH_LEAD_MS before a batch's
    expected end (moving average of batch durations), not 2 ms in, so its tasks do not sit
    out a long batch."""
    leaser.lead = 0.05
    leaser.next()
    leaser.started()
    time.sleep(0.3)  # first batch: no history, the helper leases after LEASE_PREFETCH_AFTER_MS
    leaser.finished()
    t_first = FakeCtl.log[1][1]
    assert leaser.next()[0] == "L1"
    leaser.started()
    t0 = time.monotonic()
    assert t_first - (t0 - 0.3) < 0.1
    time.sleep(0.35)
    leaser.finished()
    assert [n for n, _ in FakeCtl.log] == ["MainThread", "atpu-leaser", "atpu-leaser"]
    lag = FakeCtl.log[2][1] - t0  # the second batch's lease ahead: ~0.3 - 0.05 s in
    assert 0.2 < lag < 0.32, lag
    assert leaser.pending() == [("L2", [{"id": "2"}])]


def test_short_batches_stay_serial(leaser):
    for i in range(3):
        assert leaser.next()[0] == f"L{i}"
        leaser.started()
        leaser.finished()  # sub-millisecond batch: the helper never fires
    time.sleep(0.05)
    assert [n for n, _ in FakeCtl.log] == ["MainThread"] * 3 and leaser.pending() == []


def test_stop_hands_back_the_lease_taken_ahead(leaser):
    leaser.next()
    leaser.started()
    time.sleep(0.1)
    leaser.finished()
    leaser.stop()
    assert leaser.take_ahead()[0] == "L1" and leaser.take_ahead() is None


def test_rank_lost_fails_the_lease_taken_ahead(monkeypatch):
    """a job raising RankLost ends the loop; the lease the helper took ahead is
    posted ``failed`` (RankLost) instead of being run on the broken DP group."""
    import app
    from agent_tpu_amd.parallel.watchdog import RankLost

    posted, ran = [], []

    class Ctl(FakeCtl):
        def result(self, lease_id, job_id, epoch, status, result, error, attempts_done=0):
            posted.append((lease_id, job_id, epoch, status, error and error["type"]))

    monkeypatch.setattr(app, "Controller", Ctl)
    monkeypatch.setattr(app, "IDLE_SLEEP_SEC", 0.0)
    monkeypatch.setattr(app, "_running", True)
    monkeypatch.setenv("LEASE_PREFETCH_AFTER_MS", "5")
    FakeCtl.log = []
    FakeCtl.queue = [("L0", [{"id": "a", "op": "boom", "job_epoch": 1}]),
                     ("L1", [{"id": "b", "op": "boom", "job_epoch": 2}, {"id": "c", "op": "boom"}])]

    def boom(payload):
        ran.append(payload)
        time.sleep(0.1)  # long enough for the helper to lease L1 ahead
        raise RankLost("rank 1: lost")

    agent = object.__new__(app.Agent)
    agent.handlers, agent.caps, agent.profile = {"boom": boom}, ["boom"], {}
    agent.ctl, agent.health, agent.exit_code = Ctl(), None, 0
    agent._inflight, agent._inflight_lock = {}, threading.Lock()
    agent._deferred, agent._deferred_lines = [], []
    agent._poster, agent._leaser, agent._feeder = None, None, None
    agent._loop_prefetch()
    assert agent.exit_code == app.EXIT_RANK_LOST and len(ran) == 1
    assert posted == [("L0", "a", 1, "failed", "RankLost"), ("L1", "b", 2, "failed", "RankLost"),
                      ("L1", "c", None, "failed", "RankLost")]


def test_pipelined_poster_detects_an_http10_controller():
    """a controller answering HTTP/1.0 (Python's http.server default) closes after one
    response. The poster treats that status line as a close, switches pipelining off for good, and
    hands the unanswered (already sent) results back as one attempt made."""
    import json as _json
    import threading
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    import app

    got = []

    class H(BaseHTTPRequestHandler):  # protocol_version stays "HTTP/1.0"
        def log_message(self, *_a):
            pass

        def do_POST(self):  # noqa: N802
            n = int(self.headers.get("Content-Length", "0"))
            got.append(_json.loads(self.rfile.read(n))["job_id"])
            data = b'{"ok": true}'
            self.send_response(200)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        pp = app.PipelinedPoster(f"http://127.0.0.1:{srv.server_address[1]}", 5.0)
        items = [("L", f"j{i}", None, "succeeded", {"i": i}, None) for i in range(3)]
        rest = pp.post_many(items)
        assert got[:1] == ["j0"]
        assert pp.disabled
        assert [(it[1], n) for it, n in rest] == [("j1", 1), ("j2", 1)]
        pp.close()
    finally:
        srv.shutdown()
        srv.server_close()


def test_feeder_adaptive_limit_follows_rate_and_ttl(monkeypatch):
    """Auto in-flight depth: the sized depth until completions are measured, then what the completion
    rate finishes within INFLIGHT_TTL_FRACTION of the lease TTL, clamped to [depth/3, depth]."""
    import collections

    import app

    f = app.LeaseFeeder.__new__(app.LeaseFeeder)  # the limit rule alone (no thread)
    f.depth, f.adaptive, f.floor = 768, True, 256
    f._done_log = collections.deque()
    assert f.limit() == 768
    monkeypatch.setattr(app, "LEASE_TIMEOUT_MS", 3000)
    monkeypatch.setattr(app, "INFLIGHT_TTL_FRACTION", 0.6)
    now = [100.0]
    monkeypatch.setattr(app.time, "monotonic", lambda: now[0])
    # 396 jobs over the last second -> 396 x 3 s x 0.6 = 712 held at most
    for i in range(11):
        f._done_log.append((99.0 + i * 0.1, 36))
    assert f.limit() == 712
    # a slow device: 50 jobs/s -> 90, clamped up to the floor
    f._done_log = collections.deque((99.0 + i * 0.1, 5) for i in range(11))
    assert f.limit() == 256
    # a fast one: clamped down to the depth
    f._done_log = collections.deque((99.0 + i * 0.1, 1000) for i in range(11))
    assert f.limit() == 768
    # fixed depth (an explicit INFLIGHT_DEPTH) ignores the rate
    f.adaptive = False
    assert f.limit() == 768
