"""``csv_shard`` / ``read_csv_shard`` — read a row range of a CSV file.

Result contract identical to ``/root/reference/ops/csv_shard.py:29-103``
(``rows`` mode returns every field as a string, keyed by the header; ``count``
mode omits ``rows``; seven validation errors returned, not raised).

Difference in mechanism: the reference re-scans the file
from byte 0 on every call (O(start_row)). Here the native C++ reader
(``agent_tpu_amd/csrc/runtime/csv_index.cpp``) memory-maps the file, builds a
byte-offset row index once per (path, size, mtime) and serves any shard in
O(shard_size). Record splitting and field parsing follow the Python ``csv``
module's excel dialect so outputs are identical; blank lines are skipped like
``csv.DictReader`` does.
"""
from __future__ import annotations

import os
from typing import Any, Dict

from . import register_op

_PREFIX = "read_csv_shard"


def _err(msg: str) -> Dict[str, Any]:
    return {"ok": False, "error": f"{_PREFIX}: {msg}"}


def _unwrap(task_or_payload: Any):
    if task_or_payload is None:
        return None, _err("missing payload")
    if not isinstance(task_or_payload, dict):
        return None, _err("payload must be a dict")
    payload = task_or_payload.get("payload") if "payload" in task_or_payload else task_or_payload
    if not isinstance(payload, dict):
        return None, _err("payload must be a dict")
    return payload, None


def read_shard(payload: Any) -> Dict[str, Any]:
    payload, error = _unwrap(payload)
    if error:
        return error
    dataset_id = payload.get("dataset_id", "unknown_dataset")
    path = payload.get("source_uri")
    if not path or not isinstance(path, str):
        return _err("payload.source_uri (string) is required")
    try:
        start = int(payload.get("start_row", 0))
        size = int(payload.get("shard_size", 100))
    except Exception:
        return _err("start_row and shard_size must be integers")
    if start < 0:
        return _err("start_row must be >= 0")
    if size <= 0:
        return _err("shard_size must be > 0")
    mode = payload.get("mode", "rows")
    if mode not in ("rows", "count"):
        return _err("mode must be 'rows' or 'count'")
    if not os.path.exists(path):
        return _err(f"file not found: {path}")

    from agent_tpu_amd.io.csv import open_csv

    try:
        table = open_csv(path)
        if mode == "count":
            n = table.count_range(start, size)
            rows = None
        else:
            rows = table.dict_rows(start, size)
            n = len(rows)
    except Exception as exc:
        return _err(f"failed reading csv: {type(exc).__name__}: {exc}")

    out: Dict[str, Any] = {"ok": True, "dataset_id": dataset_id, "mode": mode,
                           "start_row": start, "end_row": start + n, "row_count": n}
    if rows is not None:
        out["rows"] = rows
    return out


register_op("read_csv_shard")(read_shard)
register_op("csv_shard")(read_shard)
