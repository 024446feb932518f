"""Streamed ``risk_accumulate`` over a CSV column (BASELINE config 5).

The reference reduces its input in one Python pass (ref ``ops/risk_accumulate.py:34-77``);
SURVEY §2.5 asks for a streaming reduce sized for 288 GB of HBM. :func:`column_stats`
reduces field ``col`` of records ``[start, start+n)`` of a :class:`CsvTable` without ever
holding the shard's values:

* GPU: ``_atpu.RiskStream`` (``csrc/runtime/risk_stream.cpp``) copies the raw record bytes
  of each chunk into one of two pinned slots (host threads), DMAs them on a side stream, and
  the device parses the field and reduces it (``csv_parse_reduce_kernel``, K13+K12), chunk
  i's copy overlapping chunk i-1's kernels. Records the device's exact fast path does not
  take (quotes, long mantissas, inf/nan, bad syntax) are parsed here with the host parser,
  which also raises the same ``could not convert string to float`` error as before.
* CPU: the same chunking with the native host parse (``extract_doubles``) into one reusable
  buffer.

Chunk size: ``worker_sizing.risk_chunk_rows`` (``RISK_CHUNK_ROWS``; 256 MiB of pinned
staging by default), so peak host memory does not depend on ``shard_size``
(``tests/contract/test_risk_stream.py``).
"""
from __future__ import annotations

import os
import threading
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .._native import native

_STREAMS: Dict[Tuple[int, int, int, int], Any] = {}
_LOCK = threading.Lock()


def _threads() -> int:
    from ..parallel.placement import host_threads

    # this rank's share of its NUMA node (parallel/placement.py), not the whole machine
    return max(1, int(os.getenv("RISK_HOST_THREADS", "0") or 0) or host_threads(16))


def gpu_min_rows() -> int:
    """Shards below this many rows reduce on the host (``RISK_GPU_MIN_VALUES``; ``RISK_DEVICE=gpu``
    forces the device)."""
    if os.getenv("RISK_DEVICE", "auto").strip().lower() == "gpu":
        return 0
    return int(os.getenv("RISK_GPU_MIN_VALUES", "1000000"))


def chunk_rows(device: Optional[torch.device] = None) -> int:
    from worker_sizing import risk_chunk_rows

    total = 0
    if device is not None and device.type == "cuda":
        total = torch.cuda.get_device_properties(device).total_memory
    return risk_chunk_rows(total)


def _stream_for(device: torch.device, rows: int):
    """One RiskStream (2 pinned + 2 device slots) per (device, chunk geometry)."""
    from worker_sizing import RISK_RECORD_BYTES

    slot_bytes = int(os.getenv("RISK_SLOT_BYTES", "0")) or min((1 << 32) - 1, rows * RISK_RECORD_BYTES)
    fb_cap = int(os.getenv("RISK_FALLBACK_CAP", "65536"))
    key = (device.index or 0, rows, slot_bytes, fb_cap)
    with _LOCK:
        rs = _STREAMS.get(key)
        if rs is None:
            with torch.cuda.device(device):
                rs = native().RiskStream(slot_bytes, rows, fb_cap)
            _STREAMS[key] = rs
        return rs


def _merge(st: Dict[str, float], vals: np.ndarray) -> None:
    if vals.size:
        st["count"] += int(vals.size)
        st["sum"] += float(vals.sum())
        st["min"] = min(st["min"], float(vals.min()))
        st["max"] = max(st["max"], float(vals.max()))


def _host_chunks(table, start: int, n: int, col: int, rows: int) -> Dict[str, float]:
    """CPU path: native parse of one chunk at a time into a reusable buffer."""
    st = {"count": 0, "sum": 0.0, "min": float("inf"), "max": float("-inf")}
    buf = np.empty(min(rows, max(n, 1)), dtype=np.float64)
    threads = _threads()
    for a in range(start, start + n, rows):
        m = min(rows, start + n - a)
        vals = buf[:m]
        table.extract_doubles_into(a, m, col, vals, threads)
        _merge(st, vals)
    return st


def column_stats(table, start: int, n: int, col: int, device: Optional[torch.device] = None,
                 rows: Optional[int] = None) -> Tuple[torch.Tensor, Dict[str, Any]]:
    """fp64 ``[count, sum, min, max]`` (CPU tensor) of field ``col`` over records
    ``[start, start+n)``, plus ``{"device", "chunks", "bytes", "host_rows"}`` details.
    Empty input gives ``[0, 0, inf, -inf]``. Raises ValueError on a non-numeric field."""
    n = max(0, min(int(n), table.num_rows - int(start)))
    if device is not None and n < gpu_min_rows():
        device = None  # a small shard: the host parse beats the stream's setup and DMA round trips
    rows = int(rows or chunk_rows(device))
    if device is not None:
        # slots sized to the shard (a power of two >= 64 Ki rows, so the cache of streams stays
        # small) instead of always the HBM-sized chunk
        rows = min(rows, 1 << max(16, (n - 1).bit_length()))
    info: Dict[str, Any] = {"device": "cpu", "chunks": 0, "bytes": 0, "host_rows": 0}
    if device is None or device.type != "cuda" or n == 0:
        st = _host_chunks(table, start, n, col, rows) if n else {"count": 0, "sum": 0.0, "min": float("inf"),
                                                                  "max": float("-inf")}
        info["chunks"] = (n + rows - 1) // rows
    else:
        rs = _stream_for(device, rows)
        with torch.cuda.device(device):
            compute = torch.cuda.current_stream(device)
            copy = _copy_stream(device)
            r = rs.run(table, int(start), n, int(col), copy.cuda_stream, compute.cuda_stream, _threads())
        info.update(device="gpu", chunks=int(r["chunks"]), bytes=int(r["bytes"]))
        if r["overflow"]:
            # more fast-path misses than the device list holds (e.g. a quoted column): host parse
            st = _host_chunks(table, start, n, col, rows)
            info["host_rows"] = n
        else:
            st = {"count": int(r["count"]), "sum": float(r["sum"]),
                  "min": float(r["min"]) if r["count"] else float("inf"),
                  "max": float(r["max"]) if r["count"] else float("-inf")}
            host_rows = r["host_rows"]
            if len(host_rows):
                # ascending: the first bad record raises, as in the single-pass host parse
                _merge(st, np.array([table.parse_double(int(i), col) for i in host_rows], dtype=np.float64))
            info["host_rows"] = int(len(host_rows))
    stats = torch.tensor([float(st["count"]), st["sum"], st["min"], st["max"]], dtype=torch.float64)
    return stats, info


_COPY: Dict[int, torch.cuda.Stream] = {}


def _copy_stream(device: torch.device) -> "torch.cuda.Stream":
    idx = device.index or 0
    s = _COPY.get(idx)
    if s is None:
        s = _COPY[idx] = torch.cuda.Stream(device)
    return s
