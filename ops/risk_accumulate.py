"""``risk_accumulate`` — streaming count/sum/mean/min/max.

Parity with ``/root/reference/ops/risk_accumulate.py:10-77`` (same output keys,
same raised ``ValueError`` messages, float64 accumulation, ``bool`` accepted as
numeric). Large ``values`` lists go through the GPU reduction kernel (K12) when
a device is present (``RISK_DEVICE=auto|gpu|cpu``). ``source_uri`` + ``field``
reduces a CSV column (native column parse). Under ``torchrun`` (DP world > 1)
the op runs on every GPU of the node: each rank reduces its shard and the
partials are combined with RCCL all-reduces
(:func:`agent_tpu_amd.parallel.dp_ops.risk_task`).

Sums are taken with ``math.fsum``-free sequential float64 addition on the CPU
path so that results are bit-identical to the reference's ``sum()``; the GPU
path accumulates in fp64 per lane and is exact to rounding order (documented in
risk_accumulate.CONTRACT.md). JSON lists (``values`` / ``items``) are converted
and reduced in ONE native pass (``_atpu.risk_stats_list``: the reference's
conversion rules via the CPython API, same sequential sum), instead of a Python
loop; ``RISK_DEVICE=gpu`` sends them through the K12 kernel instead.
"""
from __future__ import annotations

import os
import time
from typing import Any, Dict, List

from . import register_op



def to_float(value: Any) -> float:
    if isinstance(value, (int, float)):
        return float(value)
    if isinstance(value, str):
        return float(value.strip())
    raise ValueError("value must be numeric")


def _native():
    if os.getenv("RISK_NATIVE", "1").strip().lower() in ("0", "false", "no"):
        return None
    try:
        from agent_tpu_amd._native import native

        return native()
    except Exception:
        return None


def _source(payload: Dict[str, Any]):
    """(list, mode, field) after the reference's payload checks (ref :34-53)."""
    if "values" in payload:
        raw = payload.get("values")
        if not isinstance(raw, list):
            raise ValueError("payload.values must be a list")
        return raw, 0, None
    if "items" in payload:
        items = payload.get("items")
        if not isinstance(items, list):
            raise ValueError("payload.items must be a list")
        return items, 1, payload.get("field", "risk")
    raise ValueError("payload must include either 'values' or 'items'")


def gather_array(payload: Dict[str, Any]):
    """The payload's values as a float64 numpy array (native conversion when available)."""
    import numpy as np

    nat = _native()
    lst, mode, field = _source(payload)
    if nat is not None and (mode == 0 or isinstance(field, str)):
        return nat.risk_stats_list(lst, mode, field if mode else "risk", True)[4]
    return np.asarray(_gather(payload), dtype=np.float64)


def _gather(payload: Dict[str, Any]) -> List[float]:
    if "values" in payload:
        raw = payload.get("values")
        if not isinstance(raw, list):
            raise ValueError("payload.values must be a list")
        return [to_float(v) for v in raw]
    if "items" in payload:
        items = payload.get("items")
        if not isinstance(items, list):
            raise ValueError("payload.items must be a list")
        field = payload.get("field", "risk")
        out: List[float] = []
        for it in items:
            if not isinstance(it, dict):
                raise ValueError("payload.items must contain dict objects")
            if field in it:
                out.append(to_float(it[field]))
        return out
    raise ValueError("payload must include either 'values' or 'items'")


def _stats_cpu(values: List[float]) -> Dict[str, Any]:
    total = 0.0
    lo = hi = values[0]
    for v in values:
        total += v
        if v < lo:
            lo = v
        if v > hi:
            hi = v
    return {"count": len(values), "sum": total, "mean": total / len(values), "min": lo, "max": hi}


def _use_gpu(n: int) -> bool:
    """The value-list path: the device for >= RISK_GPU_MIN_VALUES values (``RISK_DEVICE=gpu``
    forces it, ``cpu`` never); the count is checked before ``torch.cuda`` is probed."""
    from agent_tpu_amd.runtime.risk import gpu_min_rows

    if os.getenv("RISK_DEVICE", "auto").strip().lower() == "cpu":
        return False
    return n >= gpu_min_rows() and _gpu_available()


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def _dp_world() -> int:
    try:
        from agent_tpu_amd.parallel.dp import world

        return world()[1]
    except Exception:
        return 1


@register_op("risk_accumulate")
def risk_accumulate(payload: Dict[str, Any]) -> Dict[str, Any]:
    t0 = time.time()
    payload = payload if payload is not None else {}
    if _dp_world() > 1:
        # node-wide DP reduce (BASELINE config 5): every rank reduces its shard
        # with K12, then two RCCL all-reduces (SUM {count,sum}, MAX {max,-min})
        from agent_tpu_amd.parallel.dp_ops import dispatch

        return dispatch("risk_accumulate", payload)
    if "source_uri" in payload:
        # streamed in chunks (agent_tpu_amd/runtime/risk.py): raw record bytes -> pinned slots ->
        # GPU parse + reduce, chunk i's copy under chunk i-1's kernels; host memory independent
        # of shard_size
        from agent_tpu_amd.ops.reduce import stats_dict
        from agent_tpu_amd.parallel.dp_ops import csv_stats

        # the device only for shards of >= RISK_GPU_MIN_VALUES rows, decided from the row index
        # before any HIP call (a small shard never creates a GPU context)
        st, info = csv_stats(payload, 0, 1)
        stats = stats_dict(st.tolist())
        if info["device"] == "gpu":
            stats["device"] = "gpu"
        stats["stream"] = {"chunks": info["chunks"], "bytes": info["bytes"], "host_rows": info["host_rows"]}
        stats["compute_time_ms"] = (time.time() - t0) * 1000.0
        return stats
    nat = _native()
    mode_env = os.getenv("RISK_DEVICE", "auto").strip().lower()
    if nat is not None and mode_env != "gpu":
        # one native pass over the JSON list: the reference's conversions, sequential float64
        # sum and comparisons (bit-identical results), no per-element Python
        lst, mode, field = _source(payload)
        if mode == 0 or isinstance(field, str):
            cnt, total, lo, hi, _ = nat.risk_stats_list(lst, mode, field if mode else "risk", False)
            if cnt == 0:
                return {"count": 0, "sum": 0.0, "mean": 0.0, "min": None, "max": None,
                        "compute_time_ms": (time.time() - t0) * 1000.0}
            return {"count": cnt, "sum": total, "mean": total / cnt, "min": lo, "max": hi,
                    "compute_time_ms": (time.time() - t0) * 1000.0}
    values = _gather(payload)
    if not values:
        return {"count": 0, "sum": 0.0, "mean": 0.0, "min": None, "max": None,
                "compute_time_ms": (time.time() - t0) * 1000.0}
    if _use_gpu(len(values)):
        from agent_tpu_amd.ops.reduce import risk_stats

        stats = risk_stats(values)
        stats["device"] = "gpu"
    else:
        stats = _stats_cpu(values)
    stats["compute_time_ms"] = (time.time() - t0) * 1000.0
    return stats
