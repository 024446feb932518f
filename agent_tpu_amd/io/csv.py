"""CSV access through the native index (``csrc/runtime/csv_index.cpp``).

:func:`open_csv` returns a cached :class:`CsvFile` per (path, size, mtime):
the row index is built once per file version and reused by every shard
request (the reference re-scanned from byte 0 on every call,
``/root/reference/ops/csv_shard.py:17-24``).
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import Any, Dict, List, Tuple

from .._native import native

_CACHE_MAX = int(os.environ.get("CSV_INDEX_CACHE", "16"))
_cache: "OrderedDict[Tuple[str, int, int], CsvFile]" = OrderedDict()
_lock = threading.Lock()


class CsvFile:
    def __init__(self, path: str):
        self.native = native().CsvTable(path)
        self.path = path

    @property
    def header(self) -> List[str]:
        return self.native.header

    @property
    def num_rows(self) -> int:
        return self.native.num_rows

    def count_range(self, start: int, n: int) -> int:
        return max(0, min(n, self.num_rows - start))

    def dict_rows(self, start: int, n: int) -> List[Dict[Any, Any]]:
        return self.native.dict_rows(start, n)


def open_csv(path: str) -> CsvFile:
    st = os.stat(path)
    key = (os.path.abspath(path), st.st_size, st.st_mtime_ns)
    with _lock:
        f = _cache.get(key)
        if f is not None:
            _cache.move_to_end(key)
            return f
    f = CsvFile(path)
    with _lock:
        _cache[key] = f
        while len(_cache) > _CACHE_MAX:
            _cache.popitem(last=False)
    return f
