"""Rank body for the multi-process DP tests (launched by torch.distributed.run).

Each scenario exercises a collective of SURVEY.md §2.7 with the gloo backend
(CPU) through the exact code the RCCL path runs. Rank 0 prints one
``RESULT {json}`` line; any assertion failure exits non-zero.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from agent_tpu_amd.parallel import dp, dp_ops  # noqa: E402


def scen_gather():
    rank, ws = dp.world()
    res = {}
    for start, n in [(0, 0), (3, 1), (10, 5), (0, 7), (100, 1001)]:
        s, k = dp.split_range(start, n, ws, rank)
        ids = torch.arange(s, s + k, dtype=torch.int32).view(-1, 1).repeat(1, 3)
        sc = torch.arange(s, s + k, dtype=torch.float32).view(-1, 1) * 0.5
        gi, gs = dp.all_gather_rows(ids, sc)
        assert gi.shape == (n, 3) and gs.shape == (n, 1), (gi.shape, n)
        assert torch.equal(gi[:, 0], torch.arange(start, start + n, dtype=torch.int32))
        assert torch.equal(gs[:, 0], torch.arange(start, start + n, dtype=torch.float32) * 0.5)
        res[f"{start}+{n}"] = int(gi.shape[0])
    return res


def scen_pack():
    from agent_tpu_amd.models.bert import config_for, init_random

    rank, _ = dp.world()
    cfg = config_for("bert-tiny")
    pack = init_random(cfg, seed=7) if rank == 0 else None
    out = dp.broadcast_pack(pack, cfg, torch.device("cpu"))
    ref = init_random(cfg, seed=7)
    assert torch.equal(out.buffer, ref.buffer)
    desc = dp.broadcast_task({"op": "x", "n": 3} if rank == 0 else None)
    assert desc == {"op": "x", "n": 3}
    return {"bytes": int(out.buffer.numel() * out.buffer.element_size())}


def scen_t5pack():
    from agent_tpu_amd.models import t5

    rank, _ = dp.world()
    cfg = t5.config_for("t5-tiny")
    pack = t5.init_random(cfg, seed=3) if rank == 0 else None
    out = dp.broadcast_pack(pack, cfg, torch.device("cpu"), builder=t5.param_specs)
    assert torch.equal(out.buffer, t5.init_random(cfg, seed=3).buffer)
    return {"ok": True}


def scen_risk():
    """Rank 0 dispatches, the others serve in worker_loop (the app.py process model)."""
    rank, ws = dp.world()
    if rank != 0:
        dp_ops.worker_loop()
        return None
    from ops.risk_accumulate import risk_accumulate

    vals = [((i * 7919) % 1000) / 7.0 - 50.0 for i in range(1003)]
    got = dp_ops.dispatch("risk_accumulate", {"values": vals})
    ref = risk_accumulate({"values": vals})
    out = {"got": got, "ref": ref}
    items = [{"risk": "1.5"}, {"other": 2}, {"risk": 3}, {"risk": True}]
    out["items"] = dp_ops.dispatch("risk_accumulate", {"items": items})
    csv_path = os.environ["DP_TEST_CSV"]
    out["csv"] = dp_ops.dispatch("risk_accumulate", {"source_uri": csv_path, "field": "risk", "start_row": 2,
                                                     "shard_size": 40})
    try:
        dp_ops.dispatch("risk_accumulate", {"values": "nope"})
        out["bad"] = None
    except Exception as exc:
        out["bad"] = f"{type(exc).__name__}: {exc}"
    out["empty"] = dp_ops.dispatch("risk_accumulate", {"values": []})
    dp_ops.shutdown_workers()
    return out


def scen_fault():
    rank, _ = dp.world()
    if rank != 0:
        dp_ops.worker_loop()
        return None
    out = {}
    try:
        dp_ops.dispatch("risk_accumulate", {"values": [1.0, 2.0, 3.0, 4.0]})
        out["err"] = None
    except RuntimeError as exc:
        out["err"] = str(exc)
    # the job after a fault still works: workers kept serving (fault fires once)
    out["after"] = dp_ops.dispatch("risk_accumulate", {"values": [1.0, 2.0]})
    dp_ops.shutdown_workers()
    return out


def scen_summarize():
    """C5: documents split over the ranks, token ids all-gathered to rank 0;
    equals the single-process batch on the same (broadcast) weights."""
    rank, ws = dp.world()
    if rank != 0:
        import ops.map_summarize  # noqa: F401  registers nothing new; same module on every rank
        dp_ops.worker_loop()
        return None
    import ops.map_summarize as ms

    words = "alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu".split()
    texts = [" ".join(words[(i + j) % len(words)] for j in range(9)) for i in range(5)]
    gen = {"num_beams": 3, "max_length": 10, "min_length": 3}
    out = {"dp": ms.handle({"texts": texts, **gen})}
    out["single_dp"] = ms.handle({"text": texts[0], **gen})  # rank 1 gets an empty shard
    eng = ms._init_engine()
    ref, _ = eng.summarize(texts, ms._gen_config(gen))
    out["ref"] = ref
    dp_ops.shutdown_workers()
    return out


def scen_shrink():
    """Elastic recovery: a device fault on rank 2 fails that job (naming rank 2),
    drops rank 2 from the DP group, and the next jobs run on ranks {0, 1}."""
    rank, ws = dp.world()
    if rank != 0:
        dp_ops.worker_loop()
        return None
    from ops.risk_accumulate import risk_accumulate

    vals = [((i * 7919) % 1000) / 7.0 - 50.0 for i in range(1003)]
    out = {}
    try:
        dp_ops.dispatch("risk_accumulate", {"values": vals})
        out["err"] = None
    except RuntimeError as exc:
        out["err"] = str(exc)
    out["members"] = dp.members()
    out["lost"] = dp.lost_ranks()
    got = dp_ops.dispatch("risk_accumulate", {"values": vals})
    ref = risk_accumulate({"values": vals})
    out["after_ok"] = got["count"] == ref["count"] and abs(got["sum"] - ref["sum"]) < 1e-9
    out["after_world"] = got["dp_world_size"]
    # a plain (non-device) failure on a survivor does not shrink the group
    try:
        dp_ops.dispatch("risk_accumulate", {"values": "bad"})
    except ValueError as exc:
        out["bad"] = str(exc)
    out["members_after_bad"] = dp.members()
    dp_ops.shutdown_workers()
    return out


def scen_classify():
    """map_classify's ``input`` and ``texts`` forms under DP (CPU engines via
    CLASSIFY_DEVICE=cpu): every rank takes part in the model load (C1), texts
    are split and all-gathered (C2), and load failures, on every rank or on
    rank 0 only, fail the job on all ranks without desynchronising the group."""
    rank, ws = dp.world()
    if rank != 0:
        dp_ops.worker_loop()
        return None
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.runtime.classify import ClassifyEngine
    from ops import map_classify as mc

    model = "bert-tiny?labels=3&batch=4&seq=32"
    out = {}
    ids = [101] + [1000 + 37 * i for i in range(20)] + [102] + [0] * 10
    out["input"] = mc.map_classify({"input": ids, "model_path": model, "topk": 3, "allow_fallback": False})
    texts = [f"row {i} " + "lorem ipsum dolor sit amet " * (i % 4) for i in range(7)]
    got = mc.map_classify({"texts": texts, "model_path": model, "topk": 2, "allow_fallback": False})
    cfg = config_for("bert-tiny", num_labels=3)
    eng = ClassifyEngine(cfg, init_random(cfg, seed=0), torch.device("cpu"), batch_rows=4, seq_len=32, topk=3)
    ref = eng.classify_texts(texts, 2)
    out["texts_world"] = got["dp_world_size"]
    out["texts_rows"] = got["row_count"]
    out["texts_idx_match"] = [[t["index"] for t in r["topk"]] for r in got["rows"]] == ref.idx.tolist()
    out["texts_score_err"] = max(abs(t["score"] - s) for r, rs in zip(got["rows"], ref.score.tolist())
                                 for t, s in zip(r["topk"], rs))
    # every rank fails the load the same way -> the op's own error type, then the fallback stub
    out["missing"] = mc.map_classify({"texts": ["x"], "model_path": "/nope/model.safetensors"})
    # rank 0 alone fails (its safetensors lacks tensors; the others only allocate): the job
    # fails on every rank before the broadcast, naming rank 0
    bad = os.environ["DP_TEST_BAD_MODEL"]
    try:
        mc.map_classify({"texts": ["x"], "model_path": bad, "allow_fallback": False})
        out["rank0_only"] = None
    except Exception as exc:
        out["rank0_only"] = f"{type(exc).__name__}: {exc}"
    # the group is still in step: the next load + job works
    again = mc.map_classify({"texts": texts[:3], "model_path": model, "topk": 2, "allow_fallback": False})
    out["again_rows"] = again["row_count"]
    dp_ops.shutdown_workers()
    return out


def main():
    scen = sys.argv[1]
    dist.init_process_group("gloo")
    try:
        res = globals()[f"scen_{scen}"]()
    finally:
        if dist.is_initialized():
            if scen not in ("risk", "fault", "summarize", "shrink", "classify"):  # worker_loop ranks already left the group
                dist.barrier()
            dist.destroy_process_group()
    if int(os.environ.get("RANK", "0")) == 0:
        print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
