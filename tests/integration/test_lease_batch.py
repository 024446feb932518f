"""Same-op jobs of one lease run as one device batch (VERDICT r2 'next' #2).

The agent runs twice against the mock controller with the same multi-task lease:
once batching (LEASE_BATCH=1, the default) and once job by job (LEASE_BATCH=0).
Every job must get its own result with its own ``job_epoch``, identical to the
job-by-job result, and a bad payload must fail (or soft-fail) only itself.
CPU only: classify runs the fp32 oracle path (CLASSIFY_DEVICE=cpu), summarize
the fp32 CPU path (SUMMARIZE_FORCE_CPU=1) on tiny random-init models.
"""
import pytest

from .mock_controller import MockController
from .test_agent_loop import start_agent, stop_agent

MODEL = "bert-tiny?labels=5&batch=4&seq=32"


def _ids(seed):
    return [101] + [1000 + (13 * i + 7 * seed) % 3000 for i in range(8 + seed)] + [102] + [0] * (22 - seed)


def _classify_jobs():
    jobs = [
        {"id": "a", "op": "map_classify", "job_epoch": 3, "payload": {"input": _ids(1), "model_path": MODEL}},
        {"id": "b", "op": "map_classify", "job_epoch": 4, "payload": {"input": _ids(2), "model_path": MODEL, "topk": 2}},
        {"id": "bad", "op": "map_classify", "payload": {"input": [1, 2, 3], "model_path": MODEL}},
        {"id": "strict", "op": "map_classify", "payload": {"input": [1, 2], "model_path": MODEL,
                                                           "allow_fallback": False}},
        {"id": "e", "op": "echo", "payload": {"k": 1}},
        {"id": "t1", "op": "map_classify", "payload": {"texts": ["alpha beta", "gamma", "delta eps zeta"],
                                                       "model_path": MODEL, "topk": 3}},
        {"id": "t2", "op": "map_classify", "payload": {"texts": ["eta theta iota kappa"] * 6, "model_path": MODEL}},
        {"id": "c", "op": "map_classify", "payload": {"input": _ids(5), "model_path": MODEL, "topk": 1}},
        # a bad ``output`` fails only its own job: texts and input forms, soft and strict
        {"id": "bo1", "op": "map_classify", "payload": {"texts": ["x y"], "model_path": MODEL, "output": "xml"}},
        {"id": "bo2", "op": "map_classify", "payload": {"input": _ids(3), "model_path": MODEL, "output": 7}},
        {"id": "bo3", "op": "map_classify", "payload": {"texts": ["x"], "model_path": MODEL, "output": "xml",
                                                        "allow_fallback": False}},
    ]
    return jobs


def _run(jobs, tasks, batch, **env):
    ctl = MockController().start()
    try:
        ctl.lease(*jobs, lease_id="LB")
        p = start_agent(ctl, tasks=tasks, LEASE_BATCH=batch, MAX_TASKS=len(jobs), CLASSIFY_DEVICE="cpu",
                        OMP_NUM_THREADS="2", **env)
        try:
            want = {j["id"] for j in jobs}
            assert ctl.wait(lambda c: want <= {r["job_id"] for r in c.results}, 240), ctl.results
        finally:
            rc, out = stop_agent(p, timeout=60)
        assert rc == 0, out[-3000:]
        return {r["job_id"]: r for r in ctl.results}, ctl.lease_requests[0]
    finally:
        ctl.stop()


def test_classify_lease_batch_matches_single():
    jobs = _classify_jobs()
    batched, lease_req = _run(jobs, "echo,map_classify", "1")
    single, _ = _run(jobs, "echo,map_classify", "0")
    assert lease_req["max_tasks"] == len(jobs)
    assert lease_req["worker_profile"]["workers"]["max_batch_tasks"] == 1024
    assert lease_req["worker_profile"]["workers"]["batch_ops"] == ["map_classify"]
    assert lease_req["worker_profile"]["limits"] == {"max_payload_bytes": 262144, "max_tokens": 2048}
    for jid in ("a", "b", "c"):
        rb, rs = batched[jid], single[jid]
        assert rb["status"] == rs["status"] == "succeeded"
        assert rb["job_epoch"] == {"a": 3, "b": 4, "c": None}[jid]
        assert set(rb["result"]) == {"op", "model_path", "topk", "elapsed_ms"}
        tb, ts = rb["result"]["topk"], rs["result"]["topk"]
        assert [t["index"] for t in tb] == [t["index"] for t in ts]
        assert all(abs(x["score"] - y["score"]) < 1e-5 for x, y in zip(tb, ts))
    assert len(batched["b"]["result"]["topk"]) == 2 and len(batched["c"]["result"]["topk"]) == 1
    # bad payloads: reference fallback stub (allow_fallback default), or a failed job
    assert batched["bad"]["result"]["fallback"] == "cpu" and batched["bad"]["result"]["topk"] == []
    assert batched["bad"]["result"]["reason"] == single["bad"]["result"]["reason"]
    assert "Input size mismatch" in batched["bad"]["result"]["reason"]
    assert batched["strict"]["status"] == "failed" and batched["strict"]["error"]["type"] == "ValueError"
    assert batched["strict"]["error"]["message"] == single["strict"]["error"]["message"]
    assert batched["e"]["result"] == {"ok": True, "echo": {"k": 1}}
    for jid in ("t1", "t2"):
        rb, rs = batched[jid]["result"], single[jid]["result"]
        assert rb["row_count"] == rs["row_count"]
        for x, y in zip(rb["rows"], rs["rows"]):
            assert x["row"] == y["row"] and [t["index"] for t in x["topk"]] == [t["index"] for t in y["topk"]]
    assert len(batched["t1"]["result"]["rows"][0]["topk"]) == 3
    for jid in ("bo1", "bo2"):
        rb, rs = batched[jid]["result"], single[jid]["result"]
        assert rb["fallback"] == "cpu" and rb["reason"] == rs["reason"], (rb, rs)
        assert "payload.output must be" in rb["reason"]
    assert batched["bo3"]["status"] == single["bo3"]["status"] == "failed"
    assert batched["bo3"]["error"]["type"] == "ValueError"
    assert batched["bo3"]["error"]["message"] == single["bo3"]["error"]["message"]


def test_summarize_lease_batch_matches_single():
    doc = "alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu "
    jobs = [
        {"id": "s1", "op": "map_summarize", "job_epoch": 9, "payload": {"text": doc * 3, "max_length": 10,
                                                                      "min_length": 3}},
        {"id": "s2", "op": "map_summarize", "payload": {"text": (doc[::-1] + " nu xi") * 2, "max_length": 10,
                                                        "min_length": 3}},
        {"id": "bad", "op": "map_summarize", "payload": {"text": "   "}},
        {"id": "s3", "op": "map_summarize", "payload": {"texts": [doc, doc * 2], "max_length": 10, "min_length": 3}},
        {"id": "s4", "op": "map_summarize", "payload": {"text": doc, "max_length": 8, "min_length": 2}},
    ]
    env = dict(SUMMARIZE_MODEL="t5-tiny", SUMMARIZE_FORCE_CPU="1")
    batched, _ = _run(jobs, "map_summarize", "1", **env)
    single, _ = _run(jobs, "map_summarize", "0", **env)
    assert batched["bad"]["result"] == single["bad"]["result"] == {"ok": False, "error": "no text provided"}
    for jid in ("s1", "s2", "s4"):
        assert batched[jid]["status"] == "succeeded"
        assert batched[jid]["result"]["summary"] == single[jid]["result"]["summary"]
    assert batched["s1"]["job_epoch"] == 9
    assert batched["s3"]["result"]["summaries"] == single["s3"]["result"]["summaries"]
    assert batched["s1"]["result"]["batched_docs"] == 4  # s1, s2, s3 x2 share the generation settings
    assert batched["s4"]["result"]["batched_jobs"] == 1


if __name__ == "__main__":
    pytest.main([__file__, "-q"])


def _run_inflight(jobs, tasks, depth, **env):
    """Every job in a lease of its own (MAX_TASKS=1, the reference's shape), in-flight mode."""
    ctl = MockController().start()
    try:
        for j in jobs:
            ctl.lease(j, lease_id="L-" + j["id"])
        p = start_agent(ctl, tasks=tasks, MAX_TASKS=1, INFLIGHT_DEPTH=depth, CLASSIFY_DEVICE="cpu",
                        OMP_NUM_THREADS="2", **env)
        try:
            want = {j["id"] for j in jobs}
            assert ctl.wait(lambda c: want <= {r["job_id"] for r in c.results}, 240), ctl.results
        finally:
            rc, out = stop_agent(p, timeout=60)
        assert rc == 0, out[-3000:]
        assert "in-flight mode" in out
        return {r["job_id"]: r for r in ctl.results}, list(ctl.events)
    finally:
        ctl.stop()


def test_classify_inflight_matches_single():
    """one job per lease, many leases held; the jobs leased meanwhile run as
    one batch, each result equal to the job-by-job run and carrying its own lease and epoch."""
    jobs = _classify_jobs()
    got, events = _run_inflight(jobs, "echo,map_classify", 32)
    single, _ = _run(jobs, "echo,map_classify", "0")
    for j in jobs:
        assert got[j["id"]]["lease_id"] == "L-" + j["id"]
        assert got[j["id"]]["job_epoch"] == j.get("job_epoch")
        assert got[j["id"]]["status"] == single[j["id"]]["status"]
    for jid in ("a", "b", "c"):
        tb, ts = got[jid]["result"]["topk"], single[jid]["result"]["topk"]
        assert [t["index"] for t in tb] == [t["index"] for t in ts]
        assert all(abs(x["score"] - y["score"]) < 1e-5 for x, y in zip(tb, ts))
    for jid in ("t1", "t2"):
        assert got[jid]["result"]["row_count"] == single[jid]["result"]["row_count"]
    assert got["bad"]["result"]["reason"] == single["bad"]["result"]["reason"]
    assert got["strict"]["status"] == "failed"
    # several leases were held at once: more than one lease was answered before the first result
    first_result = next(i for i, e in enumerate(events) if e[0] == "result")
    assert sum(1 for e in events[:first_result] if e[0] == "lease" and e[1]) > 1, events[:first_result + 1]


def test_summarize_inflight_matches_single():
    doc = "alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu "
    jobs = [
        {"id": "s1", "op": "map_summarize", "job_epoch": 9, "payload": {"text": doc * 3, "max_length": 10,
                                                                      "min_length": 3}},
        {"id": "s2", "op": "map_summarize", "payload": {"text": (doc[::-1] + " nu xi") * 2, "max_length": 10,
                                                        "min_length": 3}},
        {"id": "bad", "op": "map_summarize", "payload": {"text": "   "}},
        {"id": "s3", "op": "map_summarize", "payload": {"texts": [doc, doc * 2], "max_length": 10, "min_length": 3}},
        {"id": "s4", "op": "map_summarize", "payload": {"text": doc, "max_length": 8, "min_length": 2}},
    ]
    env = dict(SUMMARIZE_MODEL="t5-tiny", SUMMARIZE_FORCE_CPU="1")
    got, _ = _run_inflight(jobs, "map_summarize", 16, **env)
    single, _ = _run(jobs, "map_summarize", "0", **env)
    assert got["bad"]["result"] == single["bad"]["result"] == {"ok": False, "error": "no text provided"}
    for jid in ("s1", "s2", "s4"):
        assert got[jid]["status"] == "succeeded", got[jid]
        assert got[jid]["result"]["summary"] == single[jid]["result"]["summary"]
        assert got[jid]["result"]["inflight"] is True
    assert got["s1"]["job_epoch"] == 9 and got["s1"]["lease_id"] == "L-s1"
    assert got["s3"]["result"]["summaries"] == single["s3"]["result"]["summaries"]
