"""The agent's data-parallel process model end to end (CPU, gloo, 2 ranks):
``torchrun --nproc-per-node 2 app.py`` — rank 0 leases from the mock
controller and dispatches, rank 1 serves in ``dp_ops.worker_loop`` — for the
node-wide risk reduce (BASELINE config 5's collective path), with clean
SIGTERM shutdown of both ranks."""
import os
import signal
import socket
import subprocess
import sys
import time

import psutil
import pytest

from .mock_controller import MockController

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def ctl():
    c = MockController().start()
    yield c
    c.stop()


def test_dp_agent_risk_reduce_and_shutdown(ctl, tmp_path):
    csv = tmp_path / "risk.csv"
    csv.write_text("id,risk\n" + "".join(f"{i},{(i * 13 % 97) / 4.0}\n" for i in range(500)))
    vals = [1.0, 2.5, "3", True, -7.25]
    ctl.lease({"id": "v", "op": "risk_accumulate", "payload": {"values": vals}})
    ctl.lease({"id": "c", "op": "risk_accumulate", "payload": {"source_uri": str(csv), "field": "risk",
                                                               "start_row": 10, "shard_size": 300}})
    ctl.lease({"id": "bad", "op": "risk_accumulate", "payload": {"values": "nope"}})
    ctl.lease({"id": "e", "op": "echo", "payload": {"k": 1}})
    ctl.lease({"id": "after", "op": "risk_accumulate", "payload": {"values": [4.0, 6.0]}})
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="echo,risk_accumulate", IDLE_SLEEP_SEC="0.02",
               ERROR_LOG_EVERY_SEC="0", ATPU_DP_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               GPU_DISABLED="1", OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "app.py"]
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        assert ctl.wait(lambda c: "after" in {r["job_id"] for r in c.results}, 180), ctl.results
    finally:
        ranks = psutil.Process(p.pid).children(recursive=True)
        for r in ranks:  # the exact rank PIDs of this launcher
            try:
                r.send_signal(signal.SIGTERM)
            except psutil.NoSuchProcess:
                pass
        out, _ = p.communicate(timeout=120)
    res = {r["job_id"]: r for r in ctl.results}
    v = res["v"]["result"]
    assert res["v"]["status"] == "succeeded" and v["dp_world_size"] == 2
    assert v["count"] == 5 and v["sum"] == sum([1.0, 2.5, 3.0, 1.0, -7.25]) and v["min"] == -7.25 and v["max"] == 3.0
    c = res["c"]["result"]
    ref = [(i * 13 % 97) / 4.0 for i in range(10, 310)]
    assert c["count"] == 300 and abs(c["sum"] - sum(ref)) < 1e-9 and c["min"] == min(ref) and c["max"] == max(ref)
    assert res["bad"]["status"] == "failed" and res["bad"]["error"]["type"] == "ValueError"
    assert res["bad"]["error"]["message"] == "payload.values must be a list"
    assert res["e"]["result"] == {"ok": True, "echo": {"k": 1}}
    assert res["after"]["result"]["sum"] == 10.0  # the DP group survived the failed job
    assert p.returncode == 0, out[-3000:]
    assert "dp worker rank=1 ready" in out and "stopped" in out


def test_dp_agent_classify_input_first_and_device_fault(ctl):
    """under torchrun the FIRST job is a reference-form ``input``
    classify (the model load must involve every rank, or the DP group hangs),
    and a device fault on rank 1 with the default ``allow_fallback`` fails the
    job (it is not swallowed into the fallback stub), drops rank 1, and later
    jobs still run."""
    model = "bert-tiny?labels=3&batch=4&seq=32"
    ids = [101] + [1000 + 13 * i for i in range(12)] + [102] + [0] * 18
    ctl.lease({"id": "in", "op": "map_classify", "payload": {"input": ids, "model_path": model, "topk": 2}})
    ctl.lease({"id": "tx", "op": "map_classify", "payload": {"texts": ["a b c", "d e", "f"], "model_path": model}})
    ctl.lease({"id": "tx2", "op": "map_classify", "payload": {"texts": ["g h", "i"], "model_path": model}})
    ctl.lease({"id": "e", "op": "echo", "payload": {"k": 2}})
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="echo,map_classify", IDLE_SLEEP_SEC="0.02",
               ERROR_LOG_EVERY_SEC="0", ATPU_DP_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               GPU_DISABLED="1", OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1", CLASSIFY_DEVICE="cpu",
               MI355X_FAULT="rank:1:classify:1:device")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "app.py"]
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        assert ctl.wait(lambda c: "e" in {r["job_id"] for r in c.results}, 180), ctl.results
        # rank 1 left the DP group after its fault and exits on its own: let it finish
        # (a SIGTERM during interpreter teardown would be reported as a failed rank)
        for r in psutil.Process(p.pid).children(recursive=True):
            try:
                if r.environ().get("LOCAL_RANK") == "1":
                    r.wait(timeout=90)
            except (psutil.NoSuchProcess, psutil.AccessDenied):
                pass
    finally:
        for r in psutil.Process(p.pid).children(recursive=True):
            try:
                r.send_signal(signal.SIGTERM)
            except psutil.NoSuchProcess:
                pass
        out, _ = p.communicate(timeout=120)
    res = {r["job_id"]: r for r in ctl.results}
    first = res["in"]
    assert first["status"] == "succeeded", first
    assert set(first["result"]) == {"op", "model_path", "topk", "elapsed_ms"} and len(first["result"]["topk"]) == 2
    tx = res["tx"]
    assert tx["status"] == "failed", tx
    assert "rank 1" in tx["error"]["message"] and "hipError" in tx["error"]["message"]
    assert "dropped from the DP group" in tx["error"]["message"]
    tx2 = res["tx2"]
    assert tx2["status"] == "succeeded" and tx2["result"]["row_count"] == 2, tx2
    assert res["e"]["result"] == {"ok": True, "echo": {"k": 2}}
    assert p.returncode == 0, out[-3000:]


def _run_lost_rank(ctl, fault, extra_env=None, wait_s=90):
    """torchrun 2 ranks of app.py; rank 1 is SIGKILLed / hangs mid-job per ``fault``."""
    model = "bert-tiny?labels=3&batch=4&seq=32"
    ctl.lease({"id": "tx", "op": "map_classify", "job_epoch": 11,
               "payload": {"texts": ["d e f", "g", "h i"], "model_path": model}})
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="echo,map_classify", IDLE_SLEEP_SEC="0.02",
               ERROR_LOG_EVERY_SEC="0", ATPU_DP_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               GPU_DISABLED="1", OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1", CLASSIFY_DEVICE="cpu",
               MI355X_FAULT=fault, DP_COLLECTIVE_TIMEOUT="8", DP_HEARTBEAT_TIMEOUT="30")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "app.py"]
    t0 = time.time()
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        got = ctl.wait(lambda c: "tx" in {r["job_id"] for r in c.results}, wait_s)
        t_res = time.time() - t0
        out, _ = p.communicate(timeout=90)
    finally:
        if p.poll() is None:
            for r in psutil.Process(p.pid).children(recursive=True):
                try:
                    r.kill()
                except psutil.NoSuchProcess:
                    pass
            p.kill()
            p.communicate(timeout=30)
    assert got, (ctl.results, out[-3000:] if p.poll() is not None else "")
    return {r["job_id"]: r for r in ctl.results}, p.returncode, out, t_res


def test_dp_rank_killed_mid_job_fails_job_naming_rank(ctl):
    """SIGKILL rank 1 inside a classify job -> rank 0 posts ``failed`` naming
    rank 1 (not a hang until a backend timeout), then the agent exits non-zero for a restart."""
    res, rc, out, t_res = _run_lost_rank(ctl, "rank:1:classify:1:kill")
    tx = res["tx"]
    assert tx["status"] == "failed" and tx["job_epoch"] == 11, (tx, out[-3000:])
    assert "rank 1: process died" in tx["error"]["message"], (tx["error"], out[-3000:])
    assert t_res < 120, out[-3000:]
    assert rc != 0, out[-2000:]


def test_dp_rank_hung_mid_job_fails_job_naming_rank(ctl):
    """A wedged rank (alive, heartbeat running, never reaches the next collective): rank 0's
    watchdog names it after 0.8 x DP_COLLECTIVE_TIMEOUT and fails the in-flight job."""
    res, rc, out, t_res = _run_lost_rank(ctl, "rank:1:classify:1:hang")
    tx = res["tx"]
    assert tx["status"] == "failed" and tx["error"]["type"] == "RankLost", tx
    assert "rank 1: hung" in tx["error"]["message"], (tx["error"], out[-3000:])
    assert t_res < 120, out[-3000:]
    assert rc != 0, out[-2000:]
