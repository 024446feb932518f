"""Multi-process DP tests on CPU (gloo, world_size 2 and 4, 127.0.0.1).

SURVEY.md §4.4(4a): the collective shapes of the RCCL path (C1 weight
broadcast, C2 ragged all-gather, C3 risk all-reduce, C4 task descriptor,
C5 summarize token-id all-gather) and
the rank-0-leases / others-serve process model, including fault propagation
(``MI355X_FAULT``), run through ``torch.distributed.run`` like the driver's
multi-GPU bench.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(scenario, world=2, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("MI355X_FAULT", None)
    e.update({"ATPU_DP_BACKEND": "gloo", "OMP_NUM_THREADS": "1", "CUDA_VISIBLE_DEVICES": ""})
    e.update(env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(HERE, "dp_worker.py"), scenario]
    p = subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    return json.loads(line[-1][7:])


@pytest.mark.parametrize("world", [2, 4])
def test_ragged_all_gather_and_split(world):
    res = run_ranks("gather", world)
    assert res == {"0+0": 0, "3+1": 1, "10+5": 5, "0+7": 7, "100+1001": 1001}


def test_weight_broadcast_and_task_descriptor():
    assert run_ranks("pack", 2)["bytes"] > 0
    assert run_ranks("t5pack", 2) == {"ok": True}


def test_risk_allreduce_matches_cpu_op(tmp_path):
    csv = tmp_path / "r.csv"
    rows = ["id,risk"] + [f"{i},{(i * 37 % 101) / 10.0}" for i in range(60)]
    csv.write_text("\n".join(rows) + "\n")
    res = run_ranks("risk", 2, {"DP_TEST_CSV": str(csv)})
    got, ref = res["got"], res["ref"]
    for k in ("count", "min", "max"):
        assert got[k] == ref[k]
    assert abs(got["sum"] - ref["sum"]) < 1e-9 and abs(got["mean"] - ref["mean"]) < 1e-12
    assert got["dp_world_size"] == 2
    assert res["items"]["count"] == 3 and res["items"]["sum"] == 5.5
    vals = [(i * 37 % 101) / 10.0 for i in range(2, 42)]
    assert res["csv"]["count"] == 40 and abs(res["csv"]["sum"] - sum(vals)) < 1e-9
    assert res["csv"]["min"] == min(vals) and res["csv"]["max"] == max(vals)
    assert res["bad"] == "ValueError: payload.values must be a list"  # same error everywhere -> op contract
    assert res["empty"]["count"] == 0 and res["empty"]["min"] is None


def test_fault_on_one_rank_fails_job_and_workers_survive():
    res = run_ranks("fault", 2, {"MI355X_FAULT": "rank:1:risk:1"})
    assert res["err"] is not None and "rank 1" in res["err"] and "injected fault" in res["err"]
    assert "rank 0" not in res["err"]
    assert res["after"]["count"] == 2 and res["after"]["sum"] == 3.0


def test_summarize_dp_matches_single_process():
    res = run_ranks("summarize", 2, {"SUMMARIZE_MODEL": "t5-tiny", "SUMMARIZE_FORCE_CPU": "1"})
    dp, ref = res["dp"], res["ref"]
    assert dp["ok"] and dp["dp_world_size"] == 2 and len(dp["summaries"]) == 5
    assert dp["summaries"] == ref
    assert "allgather_ms" in dp["timing_ms"] and dp["model"] == "t5-tiny"
    assert res["single_dp"]["summary"] == ref[0] and "summaries" not in res["single_dp"]


def test_device_fault_shrinks_dp_world():
    """SURVEY.md §5.3 elastic recovery: rank 2's device fault fails the job that
    hit it, rank 2 leaves the DP group, and later jobs run (and shard) over the
    two healthy ranks; an ordinary op error does not shrink the group."""
    res = run_ranks("shrink", 3, {"MI355X_FAULT": "rank:2:risk:1:device"})
    assert res["err"] is not None and "rank 2" in res["err"] and "hipError" in res["err"]
    assert "dropped from the DP group" in res["err"]
    assert res["members"] == [0, 1] and res["lost"] == [2]
    assert res["after_ok"] and res["after_world"] == 2
    assert res["bad"] == "payload.values must be a list"
    assert res["members_after_bad"] == [0, 1]


def test_classify_input_and_texts_forms_under_dp(tmp_path):
    """ADVICE r1 (high/medium): the ``input``/``texts`` forms are dispatched to every
    rank (no rank-0-only collective), and model-load failures are exchanged before
    the weight broadcast (on all ranks, or on rank 0 alone) instead of hanging."""
    import torch
    from safetensors.torch import save_file

    bad = tmp_path / "partial.safetensors"
    save_file({"emb.word": torch.zeros(4, 4)}, str(bad))
    (tmp_path / "partial.safetensors.json").write_text('{"preset": "bert-tiny", "num_labels": 2}')
    res = run_ranks("classify", 2, {"CLASSIFY_DEVICE": "cpu", "DP_TEST_BAD_MODEL": str(bad)})
    inp = res["input"]
    assert set(inp) == {"op", "model_path", "topk", "elapsed_ms"} and len(inp["topk"]) == 3
    assert res["texts_world"] == 2 and res["texts_rows"] == 7
    assert res["texts_idx_match"] and res["texts_score_err"] < 1e-5
    assert res["missing"]["fallback"] == "cpu" and "GPU model not found" in res["missing"]["reason"]
    assert res["rank0_only"] is not None and res["rank0_only"].startswith("DPError: rank 0: KeyError")
    assert "rank 1" not in res["rank0_only"]
    assert res["again_rows"] == 3
