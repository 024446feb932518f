"""``map_classify`` (alias ``map_classify_tpu``) — BERT text classification on MI355X.

Replaces the reference's Edge-TPU op (``/root/reference/ops/map_classify_tpu.py``).
Three payload forms (see map_classify.CONTRACT.md):

1. reference form ``{"input": [token ids], "topk"?, "model_path"?,
   "allow_fallback"?}`` — one pre-tokenized row; returns exactly the
   reference keys ``{op, model_path, topk:[{index,score}], elapsed_ms}``, and on
   any error with ``allow_fallback`` (default True) the reference's stub
   ``{op, fallback:"cpu", reason, topk:[], elapsed_ms}`` (``:22-28,84-89``).
2. text rows ``{"texts": [...]}`` — tokenized on the GPU (K1).
3. CSV shard ``{"source_uri", "start_row", "shard_size", "text_column"?}`` —
   rows streamed from the native CSV index through pinned double buffers;
   under ``torchrun`` the shard is split over every GPU of the node and the
   per-rank top-k is all-gathered over RCCL.

``score`` is the softmax probability of the class (the reference returned raw
quantized outputs cast to float; see CONTRACT "Notes").
"""
from __future__ import annotations

import time
from typing import Any, Dict, List, Optional

from . import register_batch_op, register_op

OP_NAME = "map_classify_tpu"


def _topk_list(idx_row, score_row) -> List[Dict[str, Any]]:
    return [{"index": int(i), "score": float(s)} for i, s in zip(idx_row, score_row)]


def _fallback(payload: Dict[str, Any], reason: str, t0: float, op: str) -> Dict[str, Any]:
    return {"op": op, "fallback": "cpu", "reason": payload.get("fallback_reason", reason), "topk": [],
            "elapsed_ms": (time.time() - t0) * 1000.0}


def classify_ids(h, payload: Dict[str, Any], op: str, t0: float) -> Dict[str, Any]:
    """The reference form: one pre-tokenized row (``input``) -> reference keys."""
    import torch

    ids, n, k = _input_row(h, payload)
    res = h.engine.classify_ids(ids.view(1, -1), torch.tensor([n], dtype=torch.int32), k)
    return {"op": op, "model_path": h.model_path, "topk": _topk_list(res.idx[0].tolist(), res.score[0].tolist()),
            "elapsed_ms": (time.time() - t0) * 1000.0}


def _input_row(h, payload: Dict[str, Any]):
    """Validate one reference-form row -> (ids int32 [S], n_tokens, k); raises like :func:`classify_ids`.

    numpy, not torch: at hundreds of 1-row jobs per lease the ~5 torch CPU ops per row
    (tensor build, min, max, nonzero, cast) were ~40 us of dispatch overhead each row."""
    import numpy as np
    import torch

    k = max(1, min(int(payload.get("topk", 5)), h.cfg.num_labels))
    S = h.engine.S
    try:
        ids = np.asarray(payload["input"], dtype=np.int64)
    except (TypeError, ValueError, OverflowError) as exc:
        raise ValueError(f"input must be a list of {S} token ids: {exc}") from None
    if ids.ndim != 1 or ids.size != S:
        raise ValueError(f"Input size mismatch. Got {ids.size}, expected {S} for shape (1, {S}).")
    if int(ids.min()) < 0 or int(ids.max()) >= h.cfg.vocab_size:
        raise ValueError(f"token id out of range [0, {h.cfg.vocab_size})")
    nz = np.flatnonzero(ids)
    n = int(nz[-1]) + 1 if nz.size else 1
    return torch.from_numpy(ids.astype(np.int32)), max(1, n), k


def classify_batch(h, payloads: List[Dict[str, Any]], rank: int, ws: int) -> Optional[List[Any]]:
    """Several ``input``/``texts`` jobs of one lease as one device batch (every rank calls it).

    ``input`` rows (one pre-tokenized row per job, the reference job shape) are stacked
    into ``[n, S]`` and run through the encoder in chunks of the engine batch on rank 0;
    ``texts`` jobs are concatenated, split over the DP ranks and all-gathered (C2). Each
    job gets exactly its single-job result; a bad payload gets its own error entry."""
    import torch

    from agent_tpu_amd.parallel.dp import all_gather_rows, split_range
    from agent_tpu_amd.parallel.dp_ops import _check_errors, _err_str

    out: List[Any] = [None] * len(payloads)
    # ``output`` is validated per job before any device work, on every rank (same payloads
    # everywhere -> same outcome): a bad value fails only its own job, as in the single-job
    # path (run() -> _output_form), never the batch it was leased with
    for i, p in enumerate(payloads):
        try:
            _output_form(p)
        except Exception as exc:
            out[i] = ("err", exc)
    # ---- input form: rank 0 only (as the single-job path) ----
    rows = []
    if rank == 0:
        for i, p in enumerate(payloads):
            if "input" in p and out[i] is None:
                try:
                    rows.append((i,) + _input_row(h, p))
                except Exception as exc:
                    out[i] = ("err", exc)
        if rows:
            # a failure here (HIP fault, OOM on the stacked rows) fails the input jobs only:
            # raised out of the task it would leave the workers alone in the texts
            # section's collectives below (hang until the collective timeout)
            try:
                kmax = max(r[3] for r in rows)
                res = h.engine.classify_ids(torch.stack([r[1] for r in rows]),
                                            torch.tensor([r[2] for r in rows], dtype=torch.int32), kmax)
                idx_all, sc_all = res.idx.tolist(), res.score.tolist()
            except Exception as exc:
                for r in rows:
                    out[r[0]] = ("err", exc)
            else:
                for (i, _, _, k), ir, sr in zip(rows, idx_all, sc_all):
                    p = payloads[i]
                    out[i] = ("ok", {"op": p.get("_op", OP_NAME), "model_path": h.model_path,
                                     "topk": _topk_list(ir[:k], sr[:k]),
                                     "elapsed_ms": (time.time() - float(p.get("_t0", time.time()))) * 1000.0})
    # ---- texts form: every rank (same payloads everywhere -> same validation outcome) ----
    tjobs = []
    for i, p in enumerate(payloads):
        if "input" not in p and "texts" in p and out[i] is None:
            try:
                tjobs.append((i, check_texts(p), max(1, min(int(p.get("topk", 5)), h.cfg.num_labels))))
            except Exception as exc:
                out[i] = ("err", exc)
    if tjobs:
        texts = [t for _, ts, _ in tjobs for t in ts]
        kmax = max(k for _, _, k in tjobs)
        err, idx, sc = "", None, None
        try:
            s_r, n_r = split_range(0, len(texts), ws, rank)
            res = h.engine.classify_texts(texts[s_r:s_r + n_r], kmax)
            idx, sc = res.idx[:, :kmax].contiguous(), res.score[:, :kmax].contiguous()
        except Exception as exc:
            err = _err_str(exc)
        counts = _check_errors(err, int(idx.shape[0]) if idx is not None else 0)
        idx, sc = all_gather_rows(idx, sc, counts=counts)
        if rank == 0:
            idx, sc, pos = idx.cpu(), sc.cpu(), 0
            for i, ts, k in tjobs:
                n = len(ts)
                out[i] = ("ok", texts_result(h, idx[pos:pos + n], sc[pos:pos + n], payloads[i], ws))
                pos += n
    return out if rank == 0 else None


def check_texts(payload: Dict[str, Any]) -> List[str]:
    texts = payload["texts"]
    if not isinstance(texts, list):
        raise ValueError("payload.texts must be a list of strings")
    return ["" if t is None else str(t) for t in texts]


def _output_form(payload: Dict[str, Any]) -> str:
    form = payload.get("output", "rows")
    if form not in ("rows", "columns", "summary"):
        raise ValueError("payload.output must be 'rows', 'columns' or 'summary'")
    return form


def texts_result(h, idx, sc, payload: Dict[str, Any], dp_world: int) -> Dict[str, Any]:
    k = max(1, min(int(payload.get("topk", 5)), h.cfg.num_labels))
    extra = {"dp_world_size": dp_world} if dp_world > 1 else {}
    extra["_output"] = _output_form(payload)
    return _rows_result(h, idx[:, :k], sc[:, :k], 0, k, payload.get("_op", OP_NAME),
                        float(payload.get("_t0", time.time())), extra)


def csv_result(h, idx, sc, meta: Dict[str, Any], payload: Dict[str, Any]) -> Dict[str, Any]:
    k = max(1, min(int(payload.get("topk", 5)), h.cfg.num_labels))
    return _rows_result(h, idx[:, :k], sc[:, :k], int(meta["start_row"]), k, payload.get("_op", OP_NAME),
                        float(payload.get("_t0", time.time())),
                        {"dataset_id": payload.get("dataset_id", "unknown_dataset"),
                         "start_row": meta["start_row"], "end_row": meta["end_row"],
                         "dp_world_size": meta["world"], "timing_ms": meta["timing_ms"],
                         "_output": _output_form(payload)})


def _rows_result(h, idx, sc, start: int, k: int, op: str, t0: float, extra: Dict[str, Any]) -> Dict[str, Any]:
    """Result of a multi-row job. ``output``: ``rows`` (default; the reference's top-k
    dicts per row), ``columns`` (``index``/``score`` as [n, k] arrays) or ``summary``
    (top-1 histogram). rows / columns are JSON-encoded natively from the top-k arrays
    (``_atpu.topk_json``) and carried as :class:`RawJSON`: no per-row Python objects."""
    import torch

    from agent_tpu_amd._native import native
    from agent_tpu_amd.utils.rawjson import RawJSON

    form = extra.pop("_output", "rows")
    n = int(idx.shape[0])
    first = _topk_list(idx[0].tolist(), sc[0].tolist()) if n else []
    dt = time.time() - t0
    out = {"ok": True, "op": op, "model_path": h.model_path, "row_count": n,
           "topk": first, "elapsed_ms": dt * 1000.0,
           "rows_per_sec": (n / dt) if dt > 0 else None}
    out.update(extra)
    if form == "summary":
        counts = torch.bincount(idx[:, 0].to(torch.int64)).tolist() if n else []
        out.pop("topk", None)
        out["top1_histogram"] = {str(c): m for c, m in enumerate(counts) if m}
        return out
    ia = idx.to(torch.int32).contiguous().numpy()
    sa = sc.to(torch.float32).contiguous().numpy()
    nat = native()
    if form == "columns":
        out["k"] = k
        out["index"] = RawJSON(nat.topk_json(start, ia, sa, 1))
        out["score"] = RawJSON(nat.topk_json(start, ia, sa, 2))
    else:
        out["rows"] = RawJSON(nat.topk_json(start, ia, sa, 0))
    return out


def run_batch(payloads: List[Dict[str, Any]], op: str) -> List[Any]:
    """Batch handler: ``input``/``texts`` jobs of one lease go to the device together
    (one collective model load, one stacked forward); CSV-shard jobs (already large)
    and malformed payloads run through the single-job path. Per-job errors follow the
    single-job contract: the fallback stub when ``allow_fallback`` (default), else raised."""
    from agent_tpu_amd.parallel.dp_ops import dispatch

    t0 = time.time()
    out: List[Any] = [None] * len(payloads)
    groups: Dict[Any, List[int]] = {}
    for i, p in enumerate(payloads):
        p = p or {}
        if ("input" in p or "texts" in p) and not ("source_uri" in p and "input" not in p):
            groups.setdefault(p.get("model_path"), []).append(i)
            continue
        try:
            out[i] = ("ok", run(p, op=op))
        except Exception as exc:
            out[i] = ("err", exc)

    def settle(i: int, entry: Any) -> Any:
        p = payloads[i] or {}
        if entry[0] == "err" and p.get("allow_fallback", True) and not hard_failure(entry[1]):
            return ("ok", _fallback(p, str(entry[1]), t0, op))
        return entry

    for idxs in groups.values():
        descs = [dict(payloads[i], _op=op, _t0=t0) for i in idxs]
        try:
            res = dispatch("map_classify_batch", {"payloads": descs})
        except Exception as exc:
            res = [("err", exc)] * len(idxs)
        for i, entry in zip(idxs, res):
            out[i] = settle(i, entry)
    return out


@register_batch_op("map_classify_tpu")
def map_classify_tpu_batch(payloads: List[Dict[str, Any]]) -> List[Any]:
    return run_batch(payloads, "map_classify_tpu")


@register_batch_op("map_classify")
def map_classify_batch(payloads: List[Dict[str, Any]]) -> List[Any]:
    return run_batch(payloads, "map_classify")


def hard_failure(exc: BaseException) -> bool:
    """Failures the fallback stub must not hide: a HIP device fault (the agent
    marks the device unhealthy from the raised error), any DP job failure
    (it names the ranks; a faulted rank has already left the DP group) and a
    lost rank (dead or hung process; the agent exits for a restart)."""
    from agent_tpu_amd.parallel.dp_ops import DPError, is_device_fault
    from agent_tpu_amd.parallel.watchdog import RankLost

    return isinstance(exc, (DPError, RankLost)) or is_device_fault(str(exc))


def run(payload: Dict[str, Any], ctx: Dict[str, Any] = None, op: str = OP_NAME) -> Dict[str, Any]:
    payload = payload or {}
    t0 = time.time()
    allow_fallback = payload.get("allow_fallback", True)
    try:
        # Every form runs as a DP task: under torchrun the descriptor is
        # broadcast first, so all ranks load (and cache) the same models in the
        # same order and the C1 weight broadcast always has every rank in it.
        from agent_tpu_amd.parallel.dp_ops import dispatch

        _output_form(payload)  # validated before any device work
        if "source_uri" in payload and "input" not in payload:
            return dispatch("map_classify_csv", dict(payload, _op=op, _t0=t0))
        if "input" not in payload and "texts" not in payload:
            raise ValueError('payload missing required key: "input" (or "texts" / "source_uri")')
        return dispatch("map_classify_rows", dict(payload, _op=op, _t0=t0))
    except Exception as exc:
        if allow_fallback and not hard_failure(exc):
            return _fallback(payload, str(exc), t0, op)
        raise


@register_op("map_classify_tpu")
def map_classify_tpu(payload: Dict[str, Any], ctx: Dict[str, Any] = None) -> Dict[str, Any]:
    return run(payload, ctx, op="map_classify_tpu")


@register_op("map_classify")
def map_classify(payload: Dict[str, Any], ctx: Dict[str, Any] = None) -> Dict[str, Any]:
    return run(payload, ctx, op="map_classify")
