"""``map_summarize`` — abstractive summarisation on the encoder-decoder HIP path.

Reference: ``/root/reference/ops/map_summarize.py`` (HF BART-large-CNN on CPU,
one document per call, ``generate(num_beams=4, max_length=130, min_length=30,
early_stopping=True)``). Here: T5 (BASELINE config 4, default) or BART
(``SUMMARIZE_MODEL_FAMILY=bart``, model from the reference's ``BART_MODEL``
env, default facebook/bart-large-cnn with its generation defaults) with
random-init weights on the hand-written kernels (agent_tpu_amd/models/t5.py,
bart.py), batched beam search with HF's semantics
(agent_tpu_amd/runtime/summarize.py), documents tokenised with the same hash
tokenizer as map_classify (no SentencePiece/BPE model is available offline;
see map_summarize.CONTRACT.md).

Under ``torchrun`` (DP world > 1) the documents are split over the ranks
(contiguous shards), every rank decodes its shard with its own GPU, and the
token ids come back to rank 0 in one all-gather; the
weights reach the ranks in one RCCL broadcast of the flat pack (C1).

Output keys are the reference's ``{ok, summary, device, model}``; ``texts``
(a list) returns ``summaries``. Fix: the payload is
validated BEFORE the model is built. ``SUMMARIZE_FORCE_CPU=1`` runs the fp32
PyTorch reference path (the reference defaulted to CPU; here the GPU is the
default).
"""
from __future__ import annotations

import os
import threading
import time
from typing import Any, Dict, List, Optional

from . import register_batch_op, register_op, register_stream_op



def _resolve_model() -> str:
    fam = os.getenv("SUMMARIZE_MODEL_FAMILY", "").strip().lower()
    name = os.getenv("SUMMARIZE_MODEL", "").strip()
    if not fam:
        fam = "bart" if name.split("/")[-1].lower().startswith("bart") else "t5"
    if fam == "bart":
        return name if name.split("/")[-1].lower().startswith("bart") else os.getenv("BART_MODEL",
                                                                                      "facebook/bart-large-cnn")
    if fam != "t5":
        raise ValueError(f"SUMMARIZE_MODEL_FAMILY must be t5 or bart, got {fam!r}")
    return name if name.split("/")[-1].lower().startswith("t5") else "t5-base"


MODEL_NAME = _resolve_model()
FORCE_CPU = os.getenv("SUMMARIZE_FORCE_CPU", "0").strip().lower() in ("1", "true", "yes")
MAX_SOURCE_TOKENS = int(os.getenv("SUMMARIZE_MAX_SOURCE_TOKENS", "1024"))  # ref ops/map_summarize.py:49

_lock = threading.Lock()
_engine = None
_device = "cpu"


def _init_engine():
    global _engine, _device
    if _engine is not None:
        return _engine
    with _lock:
        if _engine is not None:
            return _engine
        import torch

        from agent_tpu_amd.runtime.summarize import SummarizeEngine, build_model

        if not FORCE_CPU and torch.cuda.is_available():
            dev = torch.device("cuda", int(os.getenv("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
        else:
            dev = torch.device("cpu")
        model, _ = build_model(MODEL_NAME, device=dev, seed=int(os.getenv("MODEL_SEED", "0")),
                               fp32=dev.type == "cpu", broadcast=_dp_world() > 1)
        eng = SummarizeEngine(model, MAX_SOURCE_TOKENS)
        _engine, _device = eng, ("cuda" if dev.type == "cuda" else "cpu")
        print(f"[map_summarize] {MODEL_NAME} ready on {_device}", flush=True)
        return _engine


def _dp_world() -> int:
    try:
        from agent_tpu_amd.parallel.dp import world

        return world()[1]
    except Exception:
        return 1


_GEN_KEYS = ("num_beams", "max_length", "min_length", "length_penalty", "no_repeat_ngram_size")


def result(texts_mode: bool, summaries: List[str], steps: int, timing_ms: Dict[str, float], t0: float,
           **extra: Any) -> Dict[str, Any]:
    out: Dict[str, Any] = {"ok": True, "device": _device, "model": MODEL_NAME,
                           "elapsed_ms": (time.time() - t0) * 1000.0, "decode_steps": steps,
                           "timing_ms": timing_ms, **extra}
    if texts_mode:
        out["summaries"] = summaries
    else:
        out["summary"] = summaries[0]
    return out


def _gen_config(payload: Dict[str, Any]):
    from agent_tpu_amd.runtime.summarize import GenConfig

    return GenConfig(num_beams=int(payload.get("num_beams", 4)), max_length=int(payload.get("max_length", 130)),
                     min_length=int(payload.get("min_length", 30)),
                     length_penalty=(float(payload["length_penalty"]) if "length_penalty" in payload else None),
                     no_repeat_ngram_size=(int(payload["no_repeat_ngram_size"])
                                           if "no_repeat_ngram_size" in payload else None),
                     early_stopping=True)


@register_op("map_summarize")
def handle(payload: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    v = _validate_one(payload)
    if isinstance(v, dict):
        return v
    texts, _, gen = v
    t0 = time.time()
    if _dp_world() > 1:
        from agent_tpu_amd.parallel.dp_ops import dispatch

        desc = {k: payload[k] for k in _GEN_KEYS if k in payload}
        desc.update(texts=texts, texts_mode="texts" in payload, t0=t0)
        return dispatch("map_summarize", desc)
    eng = _init_engine()
    summaries, res = eng.summarize(texts, gen)
    return result("texts" in payload, summaries, res.steps, res.timing_ms, t0)


def _validate_one(payload: Any):
    """-> (texts, texts_mode, gen) or an ``{"ok": False, ...}`` soft-error result (as :func:`handle`)."""
    if not payload or not isinstance(payload, dict):
        return {"ok": False, "error": "empty payload"}
    if "texts" in payload:
        raw = payload.get("texts")
        if not isinstance(raw, list) or not raw or not all(isinstance(t, str) and t.strip() for t in raw):
            return {"ok": False, "error": "payload.texts must be a non-empty list of non-empty strings"}
        texts, mode = [t.strip() for t in raw], True
    else:
        text = payload.get("text", "")
        text = text.strip() if isinstance(text, str) else ""
        if not text:
            return {"ok": False, "error": "no text provided"}
        texts, mode = [text], False
    try:
        gen = _gen_config(payload)
    except (TypeError, ValueError) as exc:
        return {"ok": False, "error": f"bad generation parameter: {exc}"}
    return texts, mode, gen


@register_batch_op("map_summarize")
def handle_batch(payloads: List[Dict[str, Any]]) -> List[Any]:
    """Several leased ``map_summarize`` jobs as ONE beam-search batch.

    The reference job stream is one document per task (ref ``ops/map_summarize.py:39-49``)
    decoded at batch 1; here the documents of every job of a lease that share the
    generation settings are decoded together (one encoder pass, one batched beam search)
    and split back per job. Beam search is per document, so each job's summary equals
    its single-job result. Invalid payloads get their own soft error."""
    out: List[Any] = [None] * len(payloads)
    groups: Dict[tuple, List[tuple]] = {}
    for i, p in enumerate(payloads):
        v = _validate_one(p)
        if isinstance(v, dict):
            out[i] = ("ok", v)
            continue
        texts, mode, gen = v
        key = (gen.num_beams, gen.max_length, gen.min_length, gen.length_penalty, gen.no_repeat_ngram_size)
        groups.setdefault(key, []).append((i, texts, mode, gen, p))
    for members in groups.values():
        t0 = time.time()
        all_texts = [t for _, texts, _, _, _ in members for t in texts]
        gen = members[0][3]
        try:
            if _dp_world() > 1:
                from agent_tpu_amd.parallel.dp_ops import dispatch

                desc = {k: members[0][4][k] for k in _GEN_KEYS if k in members[0][4]}
                desc.update(texts=all_texts, texts_mode=True, t0=t0)
                res = dispatch("map_summarize", desc)
                summaries, steps, timing = res["summaries"], res["decode_steps"], res.get("timing_ms", {})
                extra = {"dp_world_size": res.get("dp_world_size", _dp_world())}
            else:
                eng = _init_engine()
                summaries, r = eng.summarize(all_texts, gen)
                steps, timing, extra = r.steps, r.timing_ms, {}
        except Exception as exc:
            for i, *_ in members:
                out[i] = ("err", exc)
            continue
        pos = 0
        for i, texts, mode, _, _ in members:
            mine = summaries[pos:pos + len(texts)]
            pos += len(texts)
            out[i] = ("ok", result(mode, mine, steps, timing, t0, batched_docs=len(all_texts),
                                   batched_jobs=len(members), **extra))
    return out


class _InflightSummarize:
    """In-flight executor (``ops.register_stream_op``): single-document (or ``texts``) jobs join
    the running beam searches at their next decode-step boundary and complete the step their
    hypotheses are final (:class:`agent_tpu_amd.runtime.summarize.SummarizeStream`). The result
    dict is :func:`result`'s, plus the in-flight ``batched_docs`` / ``queue_ms`` details."""

    def __init__(self):
        from agent_tpu_amd.runtime.summarize import SummarizeStream

        self.stream = SummarizeStream(_init_engine())
        self.meta: Dict[Any, tuple] = {}

    def submit(self, tag: Any, payload: Any) -> Optional[tuple]:
        """Queue a job; a payload that fails validation is answered at once (its soft error)."""
        v = _validate_one(payload)
        if isinstance(v, dict):
            return ("ok", v)
        texts, mode, gen = v
        self.meta[tag] = (mode, time.time())
        try:
            self.stream.submit(tag, texts, gen)
        except Exception as exc:  # tokenization / shape errors: this job only
            self.meta.pop(tag, None)
            return ("err", exc)
        return None

    def busy(self) -> bool:
        return self.stream.busy()

    def cancel_queued(self) -> List[Any]:
        tags = self.stream.cancel_queued()
        for t in tags:
            self.meta.pop(t, None)
        return tags

    def abort(self) -> List[Any]:
        tags = self.stream.abort()
        self.meta.clear()
        return tags

    def pump(self) -> List[tuple]:
        out = []
        for tag, summaries, _, info in self.stream.pump():
            mode, t0 = self.meta.pop(tag)
            steps = info.pop("decode_steps", None)
            out.append((tag, ("ok", result(mode, summaries, steps if steps is not None else -1, {}, t0,
                                           inflight=True, **info))))
        return out


@register_stream_op("map_summarize")
def inflight_executor():
    """None under DP (a DP job is split over the ranks by ``dispatch``; no in-flight form)."""
    if _dp_world() > 1:
        return None
    return _InflightSummarize()
