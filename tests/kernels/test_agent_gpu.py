"""End to end on the GPU: the real agent (app.py) under torchrun with 2 ranks
sharing the one GPU (gloo rehearsal of the RCCL process model), leasing
map_classify CSV-shard jobs from the mock controller: C1 weight broadcast,
per-rank shard classification on the HIP path, C2 all-gather of top-k, and
the single-rank result bit-identical to the 2-rank one (batch invariance)."""
import os
import signal
import socket
import subprocess
import sys

import psutil
import pytest

from tests.integration.mock_controller import MockController

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_agent(ctl, nproc, extra_env):
    env = dict(os.environ, CONTROLLER_URL=ctl.url, TASKS="echo,map_classify", IDLE_SLEEP_SEC="0.02",
               ERROR_LOG_EVERY_SEC="0", ATPU_DP_BACKEND="gloo", PYTHONUNBUFFERED="1",
               GPU_MODEL_PATH="bert-tiny?labels=3&batch=64", HSA_ENABLE_IPC_MODE_LEGACY="0", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "app.py"]
    return subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def _stop(p):
    for r in psutil.Process(p.pid).children(recursive=True):
        try:
            r.send_signal(signal.SIGTERM)
        except psutil.NoSuchProcess:
            pass
    out, _ = p.communicate(timeout=180)
    return out


def test_dp_agent_classify_csv(gpu, tmp_path):
    from agent_tpu_amd.utils.synthetic import write_csv

    path = str(tmp_path / "rows.csv")
    write_csv(path, 500, 30)
    job = {"op": "map_classify", "payload": {"source_uri": path, "start_row": 7, "shard_size": 301, "topk": 2,
                                              "allow_fallback": False}}
    results = {}
    for nproc in (2, 1):
        ctl = MockController().start()
        try:
            ctl.lease(dict(job, id=f"n{nproc}"))
            p = _run_agent(ctl, nproc, {})
            try:
                ok = ctl.wait(lambda c: len(c.results) >= 1, 300)
            finally:
                out = _stop(p)
            assert ok, out[-3000:]
            results[nproc] = ctl.results[0]
        finally:
            ctl.stop()
    r2, r1 = results[2]["result"], results[1]["result"]
    assert results[2]["status"] == "succeeded", results[2]
    assert r2["dp_world_size"] == 2 and r1["dp_world_size"] == 1
    assert r2["row_count"] == r1["row_count"] == 301 and r2["start_row"] == 7 and r2["end_row"] == 308
    assert [x["row"] for x in r2["rows"]] == list(range(7, 308))
    for a, b in zip(r2["rows"], r1["rows"]):
        assert [t["index"] for t in a["topk"]] == [t["index"] for t in b["topk"]]
        # batch invariance (the agent's ATPU_BATCH_INVARIANT default): a rank's shard takes other
        # row counts than the single rank's batches, and every score is still bit-identical
        assert [t["score"] for t in a["topk"]] == [t["score"] for t in b["topk"]]
