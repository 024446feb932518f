"""map_classify fallback stub and map_summarize on a CPU-only agent.

map_classify: the reference's ``allow_fallback`` semantics
(``/root/reference/ops/map_classify_tpu.py:22-28,84-89``, Appendix A probe:
``fallback_reason`` overrides the real error). map_summarize: payload
validation before model init (§2.4.16) and the fp32 CPU path
(``SUMMARIZE_FORCE_CPU=1``) end to end on t5-tiny.
"""
import importlib

import pytest
import torch

from ops import map_classify as mc

pytestmark = pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only semantics")


def test_classify_fallback_stub():
    out = mc.map_classify_tpu({"input": [1, 2, 3], "topk": 3})
    assert set(out) == {"op", "fallback", "reason", "topk", "elapsed_ms"}
    assert out["op"] == "map_classify_tpu" and out["fallback"] == "cpu" and out["topk"] == []
    assert "GPU" in out["reason"]
    out = mc.map_classify({"input": [1], "fallback_reason": "forced"})
    assert out["op"] == "map_classify" and out["reason"] == "forced"
    assert mc.map_classify_tpu(None)["fallback"] == "cpu"
    with pytest.raises(RuntimeError):
        mc.map_classify({"input": [1], "allow_fallback": False})


@pytest.fixture
def summarize(monkeypatch):
    monkeypatch.setenv("SUMMARIZE_MODEL", "t5-tiny")
    monkeypatch.setenv("SUMMARIZE_FORCE_CPU", "1")
    import ops.map_summarize as ms

    ms = importlib.reload(ms)
    yield ms
    monkeypatch.undo()
    importlib.reload(ms)


def test_summarize_validation_before_init(summarize):
    ms = summarize
    assert ms.handle(None) == {"ok": False, "error": "empty payload"}
    assert ms.handle({}) == {"ok": False, "error": "empty payload"}
    assert ms.handle({"text": "   "}) == {"ok": False, "error": "no text provided"}
    assert ms.handle({"text": 5}) == {"ok": False, "error": "no text provided"}
    assert ms.handle({"texts": []})["error"] == "payload.texts must be a non-empty list of non-empty strings"
    assert ms.handle({"texts": ["ok", ""]})["ok"] is False
    assert ms.handle({"text": "x", "num_beams": "many"})["error"].startswith("bad generation parameter")
    assert ms._engine is None  # nothing above initialised the model


def test_summarize_cpu_end_to_end(summarize):
    ms = summarize
    doc = "alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu " * 4
    out = ms.handle({"text": doc, "max_length": 12, "min_length": 4})
    assert out["ok"] and out["device"] == "cpu" and out["model"] == "t5-tiny"
    assert isinstance(out["summary"], str) and 2 <= out["decode_steps"] <= 11
    outs = ms.handle({"texts": [doc, "short one"], "max_length": 10, "min_length": 3, "num_beams": 2})
    assert outs["ok"] and len(outs["summaries"]) == 2
    words = set(doc.split()) | {"short", "one"}
    for s in outs["summaries"]:
        assert all(w in words or w.startswith("<") for w in s.split())


def test_summarize_bart_family_cpu(monkeypatch):
    monkeypatch.delenv("SUMMARIZE_MODEL", raising=False)
    monkeypatch.setenv("SUMMARIZE_MODEL_FAMILY", "bart")
    monkeypatch.setenv("BART_MODEL", "bart-tiny")
    monkeypatch.setenv("SUMMARIZE_FORCE_CPU", "1")
    import ops.map_summarize as ms

    try:
        ms = importlib.reload(ms)
        assert ms.MODEL_NAME == "bart-tiny"
        doc = "one two three four five six seven eight nine ten " * 3
        out = ms.handle({"text": doc, "max_length": 14, "min_length": 5})
        assert out["ok"] and out["model"] == "bart-tiny" and isinstance(out["summary"], str)
    finally:
        monkeypatch.undo()
        importlib.reload(ms)


def test_model_resolution(monkeypatch):
    import ops.map_summarize as ms

    for env, want in [({}, "t5-base"), ({"SUMMARIZE_MODEL": "t5-small"}, "t5-small"),
                      ({"SUMMARIZE_MODEL_FAMILY": "bart"}, "facebook/bart-large-cnn"),
                      ({"SUMMARIZE_MODEL": "bart-base"}, "bart-base"),
                      ({"SUMMARIZE_MODEL_FAMILY": "bart", "BART_MODEL": "bart-large"}, "bart-large")]:
        for k in ("SUMMARIZE_MODEL", "SUMMARIZE_MODEL_FAMILY", "BART_MODEL"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        assert ms._resolve_model() == want, env


def test_word_maps_match_python_oracle():
    """The native batched reverse map equals the per-word Python oracle:
    first word producing each id, punctuation splits, >24-byte pieces, the
    64-token cap, unicode and control characters."""
    import numpy as np
    import torch

    from agent_tpu_amd.models import t5
    from agent_tpu_amd.runtime.summarize import SummarizeEngine

    cfg = t5.config_for("t5-tiny")

    class Stub:
        def __init__(self):
            self.cfg, self.device = cfg, torch.device("cpu")

        def wrap_source(self, toks):
            return list(toks) + [cfg.eos_id]

    eng = SummarizeEngine(Stub(), 64)
    long_word = "x" * 70 + "-" + "y" * 30
    texts = ["The quick, brown fox; jumps over the lazy dog's back.", "naïve café déjà-vu   tab\there",
             long_word + " " + "z" * 2000, "a\x01b c\x1fd e", "", "   ", "repeat repeat REPEAT Repeat."]
    for text, wm in zip(texts, eng.word_maps(texts)):
        oracle = eng._reverse_map(text)
        got = {int(t): wm.words[int(w)] for t, w in zip(wm.ids, wm.word_of)}
        assert got == oracle, text
        seq = sorted(oracle)[:5] + [12345 % cfg.vocab_size, cfg.eos_id]
        want = " ".join(oracle.get(t, f"<{t}>") for t in seq if t != cfg.eos_id and t != cfg.pad_id)
        assert eng.detokenize(seq, wm) == want
    assert np.asarray(eng.word_maps([""])[0].ids).size == 0


def test_encode_texts_wrapping_matches_python_reference():
    """The array-op source wrapping equals per-row Python wrapping (T5: toks </s>; BART:
    <s> toks </s>), with truncation to max_source_len, empty rows and S padded to % 8."""
    import numpy as np
    import torch

    from agent_tpu_amd import tokenizer as T
    from agent_tpu_amd.models import bart, t5
    from agent_tpu_amd.runtime.summarize import SummarizeEngine

    texts = ["The quick, brown fox; jumps over the lazy dog's back.", "", "naïve café " * 60, "a b c", "x" * 500]
    for mod, name, pre in ((t5, "t5-tiny", False), (bart, "bart-tiny", True)):
        cfg = mod.config_for(name)

        class Stub:
            def __init__(self):
                self.cfg, self.device = cfg, torch.device("cpu")

            def wrap_source(self, toks):
                return ([cfg.bos_id] if pre else []) + list(toks) + [cfg.eos_id]

        for max_src in (16, 64, 512):
            eng = SummarizeEngine(Stub(), max_src)
            ids, lens, _ = eng.encode_texts(texts, with_maps=False)
            n_sp = 2 if pre else 1
            rows = [Stub().wrap_source(T.token_ids(t.encode(), cfg.vocab_size, max_src - 1)[:max_src - n_sp])
                    for t in texts]
            S = max(8, (max(map(len, rows)) + 7) // 8 * 8)
            want = np.full((len(rows), S), cfg.pad_id, dtype=np.int32)
            for r, toks in enumerate(rows):
                want[r, :len(toks)] = toks
            assert np.array_equal(ids.numpy(), want), (name, max_src)
            assert lens.tolist() == [len(r) for r in rows]
