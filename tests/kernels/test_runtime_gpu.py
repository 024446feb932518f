"""Runtime services on a real MI355X: health check, roctx tracing switch,
map_classify op forms (reference ids form, texts, CSV shard) and the risk GPU path."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_health_check(gpu):
    from agent_tpu_amd.runtime import health

    h = health.check()
    assert h["ok"] and 0 in h["healthy"] and not h["unhealthy"], h
    d = h["devices"][0]
    assert d["arch"].startswith("gfx950") and d["hbm_total_gb"] > 200 and d["compute_units"] >= 256
    health.mark_unhealthy(0, "test")
    assert health.last()["ok"] is False and "0" not in map(str, health.last()["healthy"])
    health._unhealthy.clear()


def test_map_classify_op_forms(gpu, tmp_path, monkeypatch):
    monkeypatch.setenv("GPU_MODEL_PATH", "bert-tiny?labels=5&batch=64")
    from agent_tpu_amd.utils.synthetic import write_csv
    from ops import map_classify as mc

    out = mc.map_classify_tpu({"input": [101] + [2000 + i for i in range(30)] + [102] + [0] * 96, "topk": 3,
                               "allow_fallback": False})
    assert set(out) == {"op", "model_path", "topk", "elapsed_ms"} and out["op"] == "map_classify_tpu"
    assert len(out["topk"]) == 3 and abs(sum(t["score"] for t in out["topk"]) - 1.0) < 1.0
    assert out["topk"][0]["score"] >= out["topk"][1]["score"] >= out["topk"][2]["score"]
    bad = mc.map_classify({"input": [1, 2, 3]})
    assert bad["fallback"] == "cpu" and "Input size mismatch" in bad["reason"]
    texts = mc.map_classify({"texts": ["hello world", "", "another row of text"], "topk": 2})
    assert texts["ok"] and texts["row_count"] == 3 and len(texts["rows"][2]["topk"]) == 2
    path = str(tmp_path / "rows.csv")
    write_csv(path, 300, 40)
    csv = mc.map_classify({"source_uri": path, "start_row": 10, "shard_size": 150, "topk": 2, "timing": "device"})
    assert csv["ok"] and csv["row_count"] == 150 and csv["start_row"] == 10 and csv["end_row"] == 160
    assert csv["rows"][0]["row"] == 10 and csv["dp_world_size"] == 1
    # CSV path == texts path on the same rows (same tokenizer, same weights)
    import csv as pycsv

    with open(path, newline="") as f:
        rows = [r["text"] for r in pycsv.DictReader(f)][10:20]
    ref = mc.map_classify({"texts": rows, "topk": 2})
    for a, b in zip(csv["rows"][:10], ref["rows"]):
        assert [t["index"] for t in a["topk"]] == [t["index"] for t in b["topk"]]
        assert abs(a["topk"][0]["score"] - b["topk"][0]["score"]) < 1e-3
    summ = mc.map_classify({"source_uri": path, "start_row": 0, "shard_size": 300, "output": "summary"})
    assert sum(summ["top1_histogram"].values()) == 300 and "rows" not in summ
    tm = csv["timing_ms"]
    assert "classify_ms" in tm and "host_stager_wait_ms" in tm and "host_drain_ms" in tm
    # device time per stage from hipEvent pairs
    for k in ("device_h2d_ms", "device_tokenize_ms", "device_encoder_ms", "device_head_ms", "device_copy_out_ms",
              "device_span_ms", "device_allgather_ms", "device_d2h_ms"):
        assert k in tm and tm[k] >= 0.0, (k, tm)
    assert tm["device_encoder_ms"] > tm["device_tokenize_ms"] and tm["device_encoder_ms"] > tm["device_head_ms"]
    # the device timeline fits inside the classify wall span
    assert tm["device_span_ms"] <= tm["classify_ms"] + 1.0, tm
    compute = tm["device_tokenize_ms"] + tm["device_encoder_ms"] + tm["device_head_ms"]
    assert compute <= tm["device_span_ms"] * tm["device_overlap"] + 1.0, tm


def test_stage_timed_classify_matches_fused_graph(gpu):
    """The stage-timed replay (tokenize | encoder | head graphs with hipEvents between)
    computes exactly what the single fused graph does; serial slots: stages add up."""
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.runtime.classify import ClassifyEngine
    from agent_tpu_amd.utils.synthetic import write_csv
    from agent_tpu_amd._native import native

    cfg = config_for("bert-base", num_labels=2)
    dev = torch.device("cuda", 0)
    eng = ClassifyEngine(cfg, init_random(cfg, seed=0), dev, batch_rows=256, seq_len=128, topk=2, concurrent=False)
    import tempfile, os
    path = os.path.join(tempfile.mkdtemp(), "t.csv")
    write_csv(path, 1100, 60)
    tab = native().CsvTable(path)
    col = tab.column_index("text")
    i1, s1, st1 = eng.classify_table(tab, 0, 1100, col)
    i2, s2, st2 = eng.classify_table(tab, 0, 1100, col, stage_timing=True)
    assert torch.equal(i1, i2) and torch.equal(s1, s2)
    tm = st2.timing_ms
    stages = sum(tm[f"device_{k}_ms"] for k in ("tokenize", "encoder", "head", "copy_out"))
    assert stages <= tm["device_span_ms"] + 0.5, tm
    assert stages >= 0.5 * tm["device_span_ms"], tm  # one compute stream: the stages fill most of the span
    assert "device_h2d_ms" not in st1.timing_ms


def test_risk_gpu_path_matches_cpu(gpu, monkeypatch):
    from ops.risk_accumulate import risk_accumulate

    vals = [((i * 7919) % 100003) / 97.0 - 400.0 for i in range(200_003)]
    monkeypatch.setenv("RISK_DEVICE", "cpu")
    ref = risk_accumulate({"values": vals})
    monkeypatch.setenv("RISK_DEVICE", "gpu")
    got = risk_accumulate({"values": vals})
    assert got["device"] == "gpu" and got["count"] == ref["count"]
    assert got["min"] == ref["min"] and got["max"] == ref["max"]
    assert abs(got["sum"] - ref["sum"]) <= 1e-9 * max(1.0, abs(ref["sum"]))


def test_model_lru_hbm_budget(gpu, monkeypatch):
    import ops._gpu_runtime as rt

    monkeypatch.setenv("MODEL_LRU_SIZE", "8")
    with rt._lock:
        rt._cache.clear()
    one = rt.get_gpu_handle("bert-tiny?seed=1&batch=32")
    per = rt.cache_info()["resident_bytes"]
    monkeypatch.setenv("MODEL_LRU_GB", str(2.5 * per / 2**30))  # room for two
    rt.get_gpu_handle("bert-tiny?seed=2&batch=32")
    assert rt.cache_info()["entries"] == ["bert-tiny?seed=1&batch=32", "bert-tiny?seed=2&batch=32"]
    assert rt.get_gpu_handle("bert-tiny?seed=1&batch=32") is one  # hit refreshes recency
    rt.get_gpu_handle("bert-tiny?seed=3&batch=32")  # evicts seed=2 (least recent)
    assert rt.cache_info()["entries"] == ["bert-tiny?seed=1&batch=32", "bert-tiny?seed=3&batch=32"]
    with rt._lock:
        rt._cache.clear()


@pytest.mark.parametrize("n", [1, 7, 9, 300])
def test_small_job_bucket_graphs_match_eager(gpu, n):
    """texts / input jobs replay bucketed graphs (rows padded to a power of two);
    results equal the eager path row for row."""
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.runtime.classify import ClassifyEngine
    from agent_tpu_amd.utils.synthetic import make_text_rows

    cfg = config_for("bert-base", num_labels=5)
    pack = init_random(cfg, seed=2)
    dev = torch.device("cuda", 0)
    g_eng = ClassifyEngine(cfg, pack, dev, batch_rows=256, seq_len=128, topk=5)
    e_eng = ClassifyEngine(cfg, pack, dev, batch_rows=256, seq_len=128, topk=5, use_graph=False)
    texts = make_text_rows(n, words_per_row=40, seed=n)
    a, b = g_eng.classify_texts(texts, 3), e_eng.classify_texts(texts, 3)
    assert a.idx.shape == (n, 3) and torch.equal(a.idx, b.idx) and torch.allclose(a.score, b.score, atol=1e-6)
    g = torch.Generator().manual_seed(n)
    ids = torch.randint(1000, cfg.vocab_size, (n, 128), generator=g, dtype=torch.int32)
    lens = torch.randint(2, 129, (n,), generator=g, dtype=torch.int32)
    ids[torch.arange(128).view(1, -1) >= lens.view(-1, 1)] = 0
    a, b = g_eng.classify_ids(ids, lens, 2), e_eng.classify_ids(ids, lens, 2)
    assert torch.equal(a.idx, b.idx) and torch.allclose(a.score, b.score, atol=1e-6)
    # and the same rows through the full fp32-free forward on the device, one call
    _, ri, rs = e_eng.model.forward(ids.to(dev), lens.to(dev), 2)
    assert torch.equal(a.idx, ri.cpu())


def test_param_pack_upload(gpu):
    """ParamPack.to(cuda): bit-identical buffer and views (the weight upload of every model load)."""
    from agent_tpu_amd.models.bert import config_for, init_random

    pack = init_random(config_for("bert-tiny", num_labels=3), seed=1)
    dev = pack.to("cuda")
    assert dev.buffer.is_cuda and torch.equal(dev.buffer.cpu(), pack.buffer)
    assert all(torch.equal(dev[n].cpu(), pack[n]) for n in pack.names())


def _risk_csv(path, vals):
    with open(path, "w") as f:
        f.write("id,risk,tail\n")
        for i, v in enumerate(vals):
            f.write(f"{i},{v},t{i % 7}\n")
    return str(path)


def test_risk_stream_gpu_parse_and_chunks(gpu, tmp_path, monkeypatch):
    """K13+K12 streamed over raw CSV records (RiskStream): record-count and byte-limited
    chunks, ragged tails; count/min/max exact and the fp64 sum to rounding against the
    one-pass host parse of the same records."""
    import numpy as np

    from agent_tpu_amd._native import native
    from agent_tpu_amd.runtime import risk

    monkeypatch.setenv("RISK_DEVICE", "gpu")  # small shards too (default: >= RISK_GPU_MIN_VALUES rows)
    rng = np.random.default_rng(3)
    vals = [f"{v:.6f}" for v in rng.uniform(-1000, 1000, 250_003)]
    t = native().CsvTable(_risk_csv(tmp_path / "r.csv", vals))
    col = t.column_index("risk")
    ref_all = t.float_column(0, t.num_rows, col)
    for rows, slot_bytes in ((1 << 20, 0), (4096, 0), (70_000, 65536 * 4)):
        monkeypatch.setenv("RISK_SLOT_BYTES", str(slot_bytes))
        for start, n in ((0, 250_003), (3, 123_457), (250_000, 10)):
            st, info = risk.column_stats(t, start, n, col, gpu, rows=rows)
            ref = ref_all[start:start + n]
            c, s, lo, hi = st.tolist()
            assert info["device"] == "gpu" and info["host_rows"] == 0
            assert c == ref.size and lo == ref.min() and hi == ref.max()
            assert abs(s - ref.sum()) <= 1e-12 * np.abs(ref).sum(), (rows, start, n, s, ref.sum())
            if slot_bytes:
                assert info["chunks"] >= (info["bytes"] + slot_bytes - 1) // slot_bytes


def test_risk_stream_gpu_fallbacks_match_host(gpu, tmp_path, monkeypatch):
    """Fields the device fast path does not take (quotes, > 19 digits, inf, exponents out of
    range) are parsed on the host: every value equals the one-pass strtod parse, and a bad
    value raises the same error."""
    import numpy as np

    from agent_tpu_amd._native import native
    from agent_tpu_amd.runtime import risk

    monkeypatch.setenv("RISK_DEVICE", "gpu")
    odd = ["1e5", "-2.5E-3", " 3.5 ", "+7", ".5", "5.", "-0", "0.1234567890123456789012", '"42.5"', "inf",
           "1e400", "123456789012345678901", "9007199254740993", "1e-30", "0.000001", "00012.50"]
    vals = [odd[i % len(odd)] if i % 3 == 0 else f"{(i % 1000) / 8:.3f}" for i in range(30_000)]
    t = native().CsvTable(_risk_csv(tmp_path / "odd.csv", vals))
    col = t.column_index("risk")
    ref = t.float_column(0, t.num_rows, col)
    st, info = risk.column_stats(t, 0, t.num_rows, col, gpu, rows=5000)
    c, s, lo, hi = st.tolist()
    assert info["host_rows"] > 0 and c == ref.size and lo == ref.min() and hi == ref.max()
    assert s == ref.sum() or abs(s - ref.sum()) <= 1e-12 * np.abs(ref[np.isfinite(ref)]).sum()
    # fast-path values themselves are strtod-exact: a column of only fast-path forms
    exact = ["1e5", "-2.5E-3", " 3.5 ", "+7", ".5", "5.", "0.000001", "00012.50", "9007199254740992", "1e22"]
    t2 = native().CsvTable(_risk_csv(tmp_path / "exact.csv", exact * 100))
    st2, info2 = risk.column_stats(t2, 0, t2.num_rows, col, gpu, rows=64)
    r2 = t2.float_column(0, t2.num_rows, col)
    assert info2["host_rows"] == 0 and st2[2].item() == r2.min() and st2[3].item() == r2.max()
    bad = native().CsvTable(_risk_csv(tmp_path / "bad.csv", ["1"] * 100 + ["x1"] + ["2"] * 50 + ["y"]))
    with pytest.raises(ValueError, match="could not convert string to float: 'x1'"):
        risk.column_stats(bad, 0, bad.num_rows, col, gpu, rows=32)
    # more misses than the device list holds: the whole range is re-parsed on the host
    monkeypatch.setenv("RISK_FALLBACK_CAP", "4")
    st3, info3 = risk.column_stats(t, 0, t.num_rows, col, gpu, rows=5001)
    assert info3["host_rows"] == t.num_rows and st3[0].item() == ref.size and st3[2].item() == ref.min()


def test_risk_op_csv_streams_on_gpu(gpu, tmp_path, monkeypatch):
    from ops.risk_accumulate import risk_accumulate

    monkeypatch.setenv("RISK_DEVICE", "gpu")
    monkeypatch.setenv("RISK_CHUNK_ROWS", "20000")
    vals = [f"{(i * 7919 % 100003) / 100:.2f}" for i in range(100_000)]
    path = _risk_csv(tmp_path / "op.csv", vals)
    out = risk_accumulate({"source_uri": path, "field": "risk", "start_row": 1, "shard_size": 99_990})
    ref = risk_accumulate({"values": [float(v) for v in vals[1:99_991]]})
    assert out["device"] == "gpu" and out["stream"]["chunks"] == 5 and out["count"] == 99_990
    assert out["min"] == ref["min"] and out["max"] == ref["max"] and abs(out["sum"] - ref["sum"]) < 1e-6


def test_rand_fill_gpu_matches_host(gpu):
    """The rand_fill kernel and its CPU twin give the same bits (bf16 / fp32, ragged tails,
    split scale), and a BERT pack built on the GPU equals the host-built one."""
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.models.params import rand_fill

    for n, dt, n0 in ((1, torch.bfloat16, -1), (1000003, torch.bfloat16, 12345), (77777, torch.float32, -1),
                      (4096, torch.float32, 100)):
        h = torch.empty(n, dtype=dt)
        g = torch.empty(n, dtype=dt, device=gpu)
        rand_fill(h, 11, "t", 0.05, n0=n0, std1=0.3)
        rand_fill(g, 11, "t", 0.05, n0=n0, std1=0.3)
        assert torch.equal(g.cpu().view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                           h.view(torch.int16 if dt == torch.bfloat16 else torch.int32)), (n, dt)
    cfg = config_for("bert-base", num_labels=2)
    pg = init_random(cfg, seed=5, device=gpu)
    ph = init_random(cfg, seed=5)
    assert torch.equal(pg.buffer.cpu(), ph.buffer)


def test_classify_row_bytes_covers_the_engine(gpu):
    """worker_sizing.classify_row_bytes (what the worker profile's batch is sized by) against
    the device memory a ClassifyEngine step really takes beyond its weights: an upper bound
    that is not loose by more than 2x (bert-base, S = 128, both staging slots)."""
    from agent_tpu_amd.models.bert import config_for, init_random
    from agent_tpu_amd.runtime.classify import ClassifyEngine
    from worker_sizing import classify_row_bytes

    cfg = config_for("bert-base", num_labels=2)
    pack = init_random(cfg, seed=0, device=gpu)
    torch.cuda.synchronize()
    B = 256
    base = torch.cuda.memory_allocated(gpu)
    torch.cuda.reset_peak_memory_stats(gpu)
    eng = ClassifyEngine(cfg, pack, gpu, batch_rows=B, seq_len=128, topk=2)
    folded = eng.memory_bytes() - pack.nbytes - sum(t.numel() for t in eng.text) \
        - sum(t.numel() * 4 for t in eng.ids_s) - sum(t.numel() * 4 for t in eng.offs)
    texts = ["word " * 200] * B
    for slot in range(2):
        eng.classify_texts(texts)
    torch.cuda.synchronize()
    used = torch.cuda.max_memory_allocated(gpu) - base - folded
    est = B * classify_row_bytes("bert-base", 128, 2)
    assert used <= est and used >= est // 2, (used, est)
